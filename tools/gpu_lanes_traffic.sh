#!/bin/bash
# PMC traffic (FETCH_SIZE and WRITE_SIZE passes) and bench lines for the
# median lane-group kernels at 512 clients: config 4 (bf16, packed) and
# config 3 (fp32).  Merged into profiles/pmc_traffic.json by hand from
# gpurun_out/pmc_traffic_lanes.json.
set -o pipefail
mkdir -p gpurun_out/r03/lanes_traffic
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/lanes_traffic
run() {  # name, kernel filter, bench args...
  local name=$1 kern=$2; shift 2
  local tag=${name//[:@]/_}
  timeout -k 10 180 python3 bench.py "$@" --steps 10 --no-cpu-baseline > $O/bench_${tag}.json 2>$O/bench_${tag}.err || return 1
  cat $O/bench_${tag}.json
  local alg
  alg=$(python3 -c "import json; print(json.load(open('$O/bench_${tag}.json'))['roofline']['alg_bytes_per_step'])") || return 1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_${tag} -o b \
    -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/fetch_${tag}.log 2>&1 || return 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_${tag} -o b \
    -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/write_${tag}.log 2>&1 || return 1
  python3 tools/pmc_traffic.py --fetch $O/fetch_${tag}/b_counter_collection.csv \
    --write $O/write_${tag}/b_counter_collection.csv --key "${name}" --kernel "${kern}" \
    --alg-bytes "${alg}" --out gpurun_out/pmc_traffic_lanes.json
}
run cfg4:single:median@K512 median_pk16_lanes_kernel --config cfg4 --op median --clients 512 \
 && run cfg3:single:median@K512 median_lanes_kernel --config cfg3 --op median --clients 512 \
 && cat gpurun_out/pmc_traffic_lanes.json
