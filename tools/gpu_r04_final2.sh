#!/bin/bash
# Round 4, checkpoint: the GPU suite, smoke, the headline bench + rocprofv3,
# the counting median at config 4's 512 clients (bench line, PMC traffic
# passes, SQ pass for its VALU per wave), Krum, and the interleaved
# multi-device ingest.  Each GPU step under its own time limit.
set -o pipefail
O=gpurun_out/r04/final2
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
pmc() {  # key, kernel filter, bench args...
  local name=$1 kern=$2; shift 2
  local tag=${name//[:@]/_}
  local alg
  alg=$(python3 -c "import json; print(json.load(open('$O/bench_${tag}.json'))['roofline']['alg_bytes_per_step'])") || return 1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_${tag} -o b \
    -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/fetch_${tag}.log 2>&1 || return 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_${tag} -o b \
    -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/write_${tag}.log 2>&1 || return 1
  python3 tools/pmc_traffic.py --fetch $O/fetch_${tag}/b_counter_collection.csv \
    --write $O/write_${tag}/b_counter_collection.csv --key "${name}" --kernel "${kern}" \
    --alg-bytes "${alg}" --out $O/pmc_traffic.json
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg3 -o bench \
      -- python3 bench.py --steps 20 --no-cpu-baseline > $O/prof_cfg3.log 2>&1 \
 && timeout -k 10 300 python bench.py --op median --config cfg4 --steps 10 --no-cpu-baseline > $O/bench_cfg4_single_median_K512.json 2>> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_median -o bench \
      -- python3 bench.py --op median --config cfg4 --steps 10 --no-cpu-baseline > $O/prof_median.log 2>&1 \
 && pmc cfg4:single:median@K512 median_pk16_lanes_kernel --op median --config cfg4 \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/sq -o run \
      -- python3 bench.py --op median --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $O/sq.log 2>&1 \
 && timeout -k 10 300 python bench.py --op krum --steps 5 --warmup 2 --no-cpu-baseline > $O/krum_cfg3.json 2>> $O/bench.err \
 && timeout -k 10 600 python tools/multidev_bench.py --clients 32 --reps 4 --ingest --out $O/multidev_bench.json > $O/multidev_bench.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -2 $O/pytest_gpu.log; cat $O/smoke.log
for f in $O/bench_*.json $O/krum_cfg3.json; do python3 -c "
import json
d=json.load(open('$f')); r=d['roofline']
print('$f', d['ms_per_step'], r['kernel_ms_per_step'], r['achieved'], r['frac'], r['traffic'], (d.get('cpu_baseline') or {}).get('ms_per_aggregation'), (r.get('valu') or {}).get('frac'))
" 2>/dev/null; done
cat $O/pmc_traffic.json 2>/dev/null | grep traffic_over
grep "ingest\|host \|device " $O/multidev_bench.log
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
