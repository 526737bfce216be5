#!/bin/bash
# Round 6, session k: the streamed bit-plane median (config 4's 512 bf16 clients) measured as the
# bench reports it: the --op median line, its rocprofv3 kernel stats, PMC traffic (FETCH_SIZE and
# WRITE_SIZE in separate passes, merged by tools/pmc_traffic.py) and the SQ VALU pass
# (tools/median_valu.py), so that the line's roofline.traffic and roofline.valu describe the new
# kernel.
set -o pipefail
OUT=gpurun_out/r06/k
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--op median --config cfg4 --no-cpu-baseline"
timeout -k 10 240 python3 bench.py $B --steps 10 > $OUT/median_cfg4.json 2> $OUT/median_cfg4.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_median -o m \
  -- python3 bench.py $B --steps 10 > $OUT/prof_median.log 2>&1 || exit 1
alg=$(python3 -c "import json; print(json.load(open('$OUT/median_cfg4.json'))['roofline']['alg_bytes_per_step'])") || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch_median -o b \
  -- python3 bench.py $B --steps 3 --warmup 1 > $OUT/fetch_median.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write_median -o b \
  -- python3 bench.py $B --steps 3 --warmup 1 > $OUT/write_median.log 2>&1 || exit 1
python3 tools/pmc_traffic.py --fetch $OUT/fetch_median/b_counter_collection.csv \
  --write $OUT/write_median/b_counter_collection.csv --key "cfg4:single:median@K512" \
  --kernel median_pk16_colstream_kernel --alg-bytes "$alg" --out $OUT/pmc_traffic_k.json || exit 1
timeout -k 10 900 python3 tools/median_valu.py collect > $OUT/median_valu_collect.log 2>&1 || exit 1
python3 tools/median_valu.py merge > $OUT/median_valu.json || exit 1
find $OUT -name "*kernel_trace.csv" -size +1M -delete
cat $OUT/pmc_traffic_k.json
