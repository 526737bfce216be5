#!/bin/bash
# Where the K = 512 median kernels spend their cycles: timings (streamed and
# one cached row), one SQ counter pass and one instruction-cache pass each.
set -o pipefail
O=gpurun_out/r03/median_sq
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o 'SQC_[A-Z0-9_]*\|SQ_[A-Z0-9_]*' $O/avail.txt | sort -u > $O/sq_counters.txt || true
for c in "f32 512" "bf16 512"; do
  set -- $c
  for one in "" "--one-row"; do
    timeout -k 10 120 python tools/median_one.py --dtype $1 --K $2 $one --reps 5 >> $O/times.jsonl 2>> $O/err.log || exit 1
  done
done
cat $O/times.jsonl
pass() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n -o run \
     -- python3 tools/median_one.py --dtype $DT --K 512 $ONE --reps 1 > $O/$n.log 2>&1
}
for DT in f32 bf16; do
  for ONE in "" "--one-row"; do
    tag=${DT}${ONE:+_one}
    pass sq_$tag SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES || exit 1
  done
done
if grep -q SQC_ICACHE_MISSES $O/sq_counters.txt; then
  for DT in f32 bf16; do ONE=""; pass ic_$DT SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQ_WAVE_CYCLES || true; done
fi
python3 - <<'PY'
import csv, collections, glob, os
for d in sorted(glob.glob("gpurun_out/r03/median_sq/*/")):
    f = glob.glob(d + "**/run_counter_collection.csv", recursive=True)
    if not f:
        continue
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f[0])):
        if "median" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(os.path.basename(d.rstrip("/")), {k: round(v) for k, v in sorted(agg.items())})
PY
