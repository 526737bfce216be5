#!/bin/bash
# Round 6, session g: the fused FedOpt kernels get the small / mid2 tile tiers at shard sizes
# (A/B against the previous build, bit-identical check, whole GPU suite on the new build), then
# PMC traffic passes (FETCH_SIZE, WRITE_SIZE in separate runs) for the config-5 fused server steps
# that had none yet (AdamW, RMSprop and the six OptRepo optimizers).  Results merge into
# gpurun_out/r06/g/pmc_traffic_g.json (tools/pmc_traffic.py), then into profiles/pmc_traffic.json,
# which bench.py reads for roofline.traffic.
set -o pipefail
OUT=gpurun_out/r06/g
mkdir -p $OUT
timeout -k 10 300 python tools/ab_fused_shards.py tools/_abbuild/libfedagg_before_small_fused.so \
    fedml_amd/lib/libfedagg.so > $OUT/ab_fused_shards.txt 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 8 --backend gloo --steps 20 --nest cfg5 > $OUT/gloo8_cfg5.json 2> $OUT/gloo8_cfg5.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # optimizer, kernel filter
  local opt=$1 kern=$2 name="cfg5:single:$1"
  timeout -k 10 120 python3 bench.py --config cfg5 --fedopt $opt --steps 20 --no-cpu-baseline > $OUT/line_${opt}.json 2>/dev/null || return 1
  local alg
  alg=$(python3 -c "import json; print(json.load(open('$OUT/line_${opt}.json'))['roofline']['alg_bytes_per_step'])") || return 1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch_${opt} -o b \
    -- python3 bench.py --config cfg5 --fedopt $opt --steps 4 --warmup 1 --no-cpu-baseline > $OUT/fetch_${opt}.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write_${opt} -o b \
    -- python3 bench.py --config cfg5 --fedopt $opt --steps 4 --warmup 1 --no-cpu-baseline > $OUT/write_${opt}.log 2>&1 || return 1
  python3 tools/pmc_traffic.py --fetch $OUT/fetch_${opt}/b_counter_collection.csv \
    --write $OUT/write_${opt}/b_counter_collection.csv --key "${name}@K64" --kernel "${kern}" \
    --alg-bytes "${alg}" --out $OUT/pmc_traffic_g.json
}
run adamw AdamEpi && run rmsprop AdagradEpi \
 && run adamax OptRepoEpi && run nadam OptRepoEpi && run radam OptRepoEpi \
 && run adadelta OptRepoEpi && run asgd OptRepoEpi && run rprop OptRepoEpi
rc=$?
cat $OUT/pmc_traffic_g.json
exit $rc
