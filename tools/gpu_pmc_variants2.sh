#!/bin/bash
# PMC traffic passes (FETCH_SIZE and WRITE_SIZE, one counter block per pass)
# for the kernels added later: the packed bf16 median at config 4 and
# LightSecAgg's mod-p sum and fused reconstruction at config-3 size.  Results merge into
# profiles/pmc_traffic.json (tools/pmc_traffic.py), which bench.py reads.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, kernel filter, bench args...
  local name=$1 kern=$2; shift 2
  timeout -k 10 120 python3 bench.py "$@" --steps 20 --no-cpu-baseline > gpurun_out/pmcv_${name}.json 2>/dev/null || return 1
  local alg
  alg=$(python3 -c "import json; print(json.load(open('gpurun_out/pmcv_${name}.json'))['roofline']['alg_bytes_per_step'])") || return 1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcv_fetch_${name} -o b \
    -- python3 bench.py "$@" --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/pmcv_fetch_${name}.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcv_write_${name} -o b \
    -- python3 bench.py "$@" --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/pmcv_write_${name}.log 2>&1 || return 1
  python3 tools/pmc_traffic.py --fetch gpurun_out/pmcv_fetch_${name}/b_counter_collection.csv \
    --write gpurun_out/pmcv_write_${name}/b_counter_collection.csv --key "${name}" --kernel "${kern}" \
    --alg-bytes "${alg}" --out gpurun_out/pmc_traffic_variants2.json
}
run cfg4:single:median median_pk16_kernel --config cfg4 --op median \
 && run cfg3:single:secagg OpSumModI64 --op secagg \
 && run cfg3:single:lsa LsaEpi --op lsa
