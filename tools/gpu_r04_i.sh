#!/bin/bash
# Round 4: the counting median's per-byte search, Fibonacci (13 sums) against
# bisection (16), in one process; then the shipped (Fibonacci) kernel's tests,
# bench line and SQ pass.
set -o pipefail
O=gpurun_out/r04/i
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MEDIAN_AB_DIR=tools/_abbuild MEDIAN_AB_SHAPES=k512 MEDIAN_AB_VARIANTS="bisect=-DFEDAGG_PK16_SEARCH=0;fib=-DFEDAGG_PK16_SEARCH=1" \
  timeout -k 10 500 python tools/median_ab.py $O/median_ab_search.json > $O/median_ab.log 2>&1 \
 && timeout -k 10 600 python -u -m pytest tests/test_gpu_defense.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
 && timeout -k 10 300 python bench.py --op median --config cfg4 --steps 10 --no-cpu-baseline > $O/median_cfg4_k512.json 2> $O/bench.err \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/sq -o run \
      -- python3 bench.py --op median --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $O/sq.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
grep '^{' $O/median_ab.log
tail -2 $O/pytest.log
python3 -c "import json; d=json.load(open('$O/median_cfg4_k512.json')); r=d['roofline']; print('median', d['ms_per_step'], r['kernel_ms_per_step'], r['achieved'], r['frac'])" 2>/dev/null
python3 - <<PY
import csv, glob
f = glob.glob("$O/sq/**/run_counter_collection.csv", recursive=True)
if f:
    s = {}
    for r in csv.DictReader(open(f[0])):
        if "median" in r["Kernel_Name"]:
            s[r["Counter_Name"]] = s.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    print("VALU per wave", s.get("SQ_INSTS_VALU", 0) / max(1, s.get("SQ_WAVES", 1)), s)
PY
exit $rc
