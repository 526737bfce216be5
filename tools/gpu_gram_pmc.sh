#!/bin/bash
# One SQ counter pass (8 SQ slots) over the centred-Gram Krum kernel at
# config 3: where its waves spend their cycles and how busy the matrix cores are.
set -o pipefail
O=gpurun_out/r03/gram_pmc2
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $O/sq -o bench \
    -- python3 bench.py --op krum --steps 2 --warmup 1 --no-cpu-baseline > $O/sq.log 2>&1
rc=$?
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/r03/gram_pmc2/sq/bench_counter_collection.csv")))
agg = collections.defaultdict(list)
for r in rows:
    if "pairgram" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, len(v), sum(v) / len(v))
PY
exit $rc
