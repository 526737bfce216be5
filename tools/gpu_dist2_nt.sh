#!/bin/bash
# dist2: non-temporal vs plain client-row loads (timings interleaved, then
# one FETCH_SIZE pass per variant).  Builds the variants on the box.
set -o pipefail
O=gpurun_out/r03/dist2_nt
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export ROBUST_VARIANTS="dxnt=-DFEDAGG_DIST2_X_NT=true;dxplain=-DFEDAGG_DIST2_X_NT=false"
timeout -k 10 300 python tools/robust_variants.py --build > $O/build.log 2>&1 || { tail -5 $O/build.log; exit 1; }
timeout -k 10 300 python tools/robust_variants.py --rounds 15 > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
for t in dxnt dxplain; do
  f=$([ $t = dxnt ] && echo true || echo false)
  ROBUST_VARIANTS="$t=-DFEDAGG_DIST2_X_NT=$f" ROBUST_NO_SHIPPED=1 \
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$t -o run \
    -- python3 tools/robust_variants.py --rounds 2 > $O/fetch_$t.log 2>&1 || { tail -5 $O/fetch_$t.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
O = "gpurun_out/r03/dist2_nt"
out = {}
for t in ("dxnt", "dxplain"):
    f = glob.glob(f"{O}/fetch_{t}/**/run_counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE" and ("dist2" in r["Kernel_Name"] or "clip" in r["Kernel_Name"]):
            per[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
    out[t] = {k: [round(x) for x in v] for k, v in per.items()}
json.dump(out, open(f"{O}/fetch_summary.json", "w"), indent=1)
print(json.dumps(out))
PY
find $O -name '*.csv' -size +2M -delete
