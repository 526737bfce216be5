#!/bin/bash
# Round 5: HBM traffic (PMC, separate FETCH_SIZE / WRITE_SIZE passes) of the
# kernels that changed this round: config 4's bf16 chain (U1V8), its fp32
# accumulation, config 5's capped SGD, config 3's MPI order.  Each pass's
# counter CSV is cut down to the measured kernel's rows.
set -o pipefail
O=gpurun_out/r05/ag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
pass() {  # name counter kernel-substring args...
  local n=$1 c=$2 k=$3; shift 3
  [ $ok = 0 ] || return
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/tmp_${n}_$c -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline "$@" > $O/${n}_$c.log 2>&1 || { ok=1; echo "FAILED $n $c"; tail -5 $O/${n}_$c.log; }
  f=$(find $O/tmp_${n}_$c -name '*counter_collection.csv' | head -1)
  if [ -n "$f" ]; then
    python3 - "$f" "$k" "$O/${n}_$c.csv" <<'PY'
import csv, sys
src, k, dst = sys.argv[1:4]
rows = list(csv.DictReader(open(src)))
keep = [r for r in rows if k in r.get("Kernel_Name", "")]
with open(dst, "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=list(rows[0].keys()) if rows else ["none"])
    w.writeheader(); w.writerows(keep)
print(dst, len(keep), "rows of", len(rows))
PY
  else
    echo "no counter csv for $n $c"
  fi
  rm -rf $O/tmp_${n}_$c
}
for c in FETCH_SIZE WRITE_SIZE; do
  pass cfg4 $c OpBF16Ref --config cfg4
  pass cfg4acc32 $c OpBF16Acc32 --config cfg4 --acc fp32
  pass cfg5sgd $c SgdEpi --config cfg5 --fedopt sgd
  pass cfg3mpi $c OpF32MulDiv --config cfg3 --op mpi
done
exit $ok
