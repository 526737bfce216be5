#!/bin/bash
# Non-temporal vs plain loads in the median lane-group kernels (half-line
# reads per wave instruction): interleaved timings, then one FETCH_SIZE pass
# per variant on the 4M-column shapes.
set -o pipefail
O=gpurun_out/r03/lanes_nt
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MEDIAN_AB_SHAPES=lanes
V="nt=-DFEDAGG_LANES_NT=1;plain=-DFEDAGG_LANES_NT=0"
MEDIAN_AB_VARIANTS="$V" timeout -k 10 300 python tools/median_ab.py $O/ab.json > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
cat $O/ab.log
for t in nt plain; do
  f=$([ $t = nt ] && echo 1 || echo 0)
  MEDIAN_AB_VARIANTS="$t=-DFEDAGG_LANES_NT=$f" MEDIAN_AB_MAXN=5000000 MEDIAN_AB_REPS=3 \
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$t -o run \
    -- python3 tools/median_ab.py $O/pmc_$t.json > $O/fetch_$t.log 2>&1 || { tail -5 $O/fetch_$t.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
O = "gpurun_out/r03/lanes_nt"
out = {}
for t in ("nt", "plain"):
    f = glob.glob(f"{O}/fetch_{t}/**/run_counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE" and "median" in r["Kernel_Name"]:
            per[r["Kernel_Name"][:90]].append(float(r["Counter_Value"]))
    out[t] = {k: [round(x) for x in v] for k, v in per.items()}
json.dump(out, open(f"{O}/fetch_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
