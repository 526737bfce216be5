#!/bin/bash
# Round 4: SQ counters of the shipped split Gram (8-wave kernel): LDS
# instructions, bank conflicts, waits, MFMA busy.
set -o pipefail
O=gpurun_out/r04/aa
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/sq1 -o run \
    -- python3 bench.py --op krum --steps 2 --warmup 1 --no-cpu-baseline > $O/sq1.log 2>&1 \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY \
    SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/sq2 -o run \
    -- python3 bench.py --op krum --steps 2 --warmup 1 --no-cpu-baseline > $O/sq2.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
python3 - <<PY
import csv, glob, json
out = {}
for d in ("sq1", "sq2"):
    f = glob.glob("$O/%s/**/run_counter_collection.csv" % d, recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        if "pairgram" in r["Kernel_Name"]:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0) + float(r["Counter_Value"]) / 3
print(json.dumps(out, indent=0))
json.dump(out, open("$O/gram_sq_per_launch.json", "w"), indent=1)
PY
exit $rc
