#!/bin/bash
# LDS counters of the radix-select median probe (fp32 K = 512 and bf16 K = 512).
set -o pipefail
O=gpurun_out/r03/rsel_pmc
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 0 2; do
  RSEL_VARIANTS=$v RSEL_REPS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS \
      SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
      --kernel-trace --output-format csv -d $O/v$v -o run -- python3 tools/median_rsel_probe.py $O/v$v.json \
      > $O/v$v.log 2>&1 || { tail -5 $O/v$v.log; exit 1; }
done
python3 - <<'PY'
import csv, collections, glob
for v in (0, 2):
    f = glob.glob(f"gpurun_out/r03/rsel_pmc/v{v}/**/run_counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        n = r["Kernel_Name"]
        key = "rsel" if "rsel" in n else ("shipped" if "median" in n else None)
        if key:
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in agg.items():
        print(v, k, {c: round(x) for c, x in sorted(d.items())})
PY
find $O -name '*.csv' -size +2M -delete
