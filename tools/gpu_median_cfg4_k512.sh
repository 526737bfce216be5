#!/bin/bash
# Config 4's median at its real client count on one GPU (512 x ViT-B/16 bf16,
# the packed lane-group kernel): bench line, rocprofv3 kernel stats, and
# FETCH_SIZE / WRITE_SIZE passes (separate runs) for the traffic check.
set -o pipefail
O=gpurun_out/cfg4k512
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --op median --config cfg4 --clients 512 --no-cpu-baseline"
timeout -k 10 300 python $B --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench \
      -- python3 $B --steps 5 --warmup 1 > $O/prof.log 2>&1 \
 && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o bench \
      -- python3 $B --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1 \
 && timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o bench \
      -- python3 $B --steps 2 --warmup 1 > $O/pmc_write.log 2>&1
rc=$?
cat $O/bench.json
exit $rc
