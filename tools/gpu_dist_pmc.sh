#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of the distance-defense
# kernels at config 3, and rocprofv3 kernel stats of the krum / dist2 / clip
# bench commands.  Every GPU step has its own time limit; the chain stops at
# the first failure.
set -o pipefail
O=gpurun_out/${1:-r02p}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --no-cpu-baseline"
ok=0
for op in dist2 clip; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${op}_${c} -o bench \
      -- python3 $B --op $op --steps 3 --warmup 1 > $O/pmc_${op}_${c}.log 2>&1 || { ok=1; break 2; }
  done
done
[ $ok -eq 0 ] && for op in krum dist2 clip; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$op -o bench \
    -- python3 $B --op $op --steps 5 --warmup 1 > $O/prof_$op.log 2>&1 || { ok=1; break; }
done
exit $ok
