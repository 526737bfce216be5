#!/bin/bash
# dist2 chunk table: run-start cuts vs absolute cuts (timings, FETCH_SIZE per
# table), then the bench line and PMC traffic of --op dist2 as shipped.
set -o pipefail
O=gpurun_out/r03/dist2_chunks
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/dist2_chunks_ab.py --rounds 20 > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
for m in run absolute; do
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$m -o run \
    -- python3 tools/dist2_chunks_ab.py --rounds 2 --only $m > $O/fetch_$m.log 2>&1 || { tail -5 $O/fetch_$m.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, json, statistics
O = "gpurun_out/r03/dist2_chunks"
out = {}
for m in ("run", "absolute"):
    f = glob.glob(f"{O}/fetch_{m}/**/run_counter_collection.csv", recursive=True)[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
         if r["Counter_Name"] == "FETCH_SIZE" and "dist2_kernel" in r["Kernel_Name"]]
    out[m] = {"FETCH_SIZE_KiB": v, "read_bytes_x2": 2 * 1024 * statistics.median(v)}
json.dump(out, open(f"{O}/fetch_summary.json", "w"), indent=1)
print(json.dumps(out))
PY
run() {  # name, kernel filter, bench args...
  local name=$1 kern=$2; shift 2
  local tag=${name//[:@]/_}
  timeout -k 10 180 python3 bench.py "$@" --steps 20 --no-cpu-baseline > $O/bench_${tag}.json 2>$O/bench_${tag}.err || return 1
  cat $O/bench_${tag}.json
  local alg
  alg=$(python3 -c "import json; print(json.load(open('$O/bench_${tag}.json'))['roofline']['alg_bytes_per_step'])") || return 1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/bfetch_${tag} -o b \
    -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/bfetch_${tag}.log 2>&1 || return 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/bwrite_${tag} -o b \
    -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/bwrite_${tag}.log 2>&1 || return 1
  python3 tools/pmc_traffic.py --fetch $O/bfetch_${tag}/b_counter_collection.csv \
    --write $O/bwrite_${tag}/b_counter_collection.csv --key "${name}" --kernel "${kern}" \
    --alg-bytes "${alg}" --out gpurun_out/pmc_traffic_dist2.json
}
run cfg3:single:dist2 dist2_kernel --op dist2 && cat gpurun_out/pmc_traffic_dist2.json
rc=$?
find $O -name '*kernel_trace.csv' -delete
find $O -name '*.csv' -size +2M -delete
exit $rc
