#!/bin/bash
# Round 4: the counting median (v_sad_u8 bisection) for packed 16-bit lane
# groups.  Median GPU tests, the A/B against the sorting networks in one
# process (bit-identical outputs required), the config-4 bench line at 512
# clients and one SQ pass for its executed VALU per wave.
set -o pipefail
O=gpurun_out/r04/b
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_defense.py -x -q --timeout 120 --timeout-method thread > $O/pytest_median.log 2>&1 \
 && MEDIAN_AB_DIR=tools/_abbuild MEDIAN_AB_VARIANTS="count=-DFEDAGG_PK16_COUNT=1;net=-DFEDAGG_PK16_COUNT=0" \
    MEDIAN_AB_SHAPES=k512 timeout -k 10 400 python tools/median_ab.py $O/median_ab_count.json > $O/median_ab.log 2>&1 \
 && timeout -k 10 300 python bench.py --op median --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline > $O/median_cfg4_k512.json 2> $O/bench.err \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/sq -o run \
      -- python3 bench.py --op median --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $O/sq.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -3 $O/pytest_median.log
cat $O/median_ab.log | grep '^{'
cat $O/median_cfg4_k512.json
python3 - <<EOF
import csv, glob
f = glob.glob("$O/sq/**/run_counter_collection.csv", recursive=True)
if f:
    s = {}
    for r in csv.DictReader(open(f[0])):
        if "median" in r["Kernel_Name"]:
            s[r["Counter_Name"]] = s.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    print("VALU per wave", s.get("SQ_INSTS_VALU", 0) / max(1, s.get("SQ_WAVES", 1)), s)
EOF
exit $rc
