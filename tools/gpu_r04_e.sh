#!/bin/bash
# Round 4: Gram timing diagnostics (MFMA phase alone / staging alone), the
# pack pool against round 3's per-call threads in the multi-device ingest,
# and the shipped counting median (4 SAD chains): tests, bench line, SQ pass.
set -o pipefail
O=gpurun_out/r04/e
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GRAM_AB_DIR=tools/_abbuild timeout -k 10 300 python tools/gram_variants.py --rounds 7 --out $O/gram_diag.json \
    --variant "nocompute=-DFEDAGG_GRAM_DIAG=1" --variant "nostage=-DFEDAGG_GRAM_DIAG=2" > $O/gram_diag.log 2>&1 \
 && FEDAGG_PACK_SPAWN=1 timeout -k 10 400 python tools/multidev_bench.py --clients 32 --reps 3 --out $O/multidev_spawn.json > $O/multidev_spawn.log 2>&1 \
 && timeout -k 10 400 python tools/multidev_bench.py --clients 32 --reps 3 --out $O/multidev_pool.json > $O/multidev_pool.log 2>&1 \
 && timeout -k 10 600 python -u -m pytest tests/test_gpu_defense.py tests/test_gpu_multidev.py tests/test_gpu_cross_silo.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
 && timeout -k 10 300 python bench.py --op median --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline > $O/median_cfg4_k512.json 2> $O/bench.err \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/sq -o run \
      -- python3 bench.py --op median --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $O/sq.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
cat $O/gram_diag.log | grep ms
grep "host\|device" $O/multidev_spawn.log $O/multidev_pool.log
tail -2 $O/pytest.log
python3 -c "import json; d=json.load(open('$O/median_cfg4_k512.json')); r=d['roofline']; print('median', d['ms_per_step'], r['kernel_ms_per_step'], r['achieved'], r['frac'], r['traffic'])" 2>/dev/null
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
