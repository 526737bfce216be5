#!/bin/bash
# Round 4: one SQ counter pass over the split-bf16 Gram (bench.py --op krum).
set -o pipefail
O=gpurun_out/r04/p
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq -o run \
    -- python3 bench.py --op krum --steps 2 --warmup 1 --no-cpu-baseline > $O/sq.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
python3 - <<PY
import csv, glob
f = glob.glob("$O/sq/**/run_counter_collection.csv", recursive=True)
if f:
    s, n = {}, {}
    for r in csv.DictReader(open(f[0])):
        if "pairgram" in r["Kernel_Name"]:
            s[r["Counter_Name"]] = s.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    print(s)
PY
exit $rc
