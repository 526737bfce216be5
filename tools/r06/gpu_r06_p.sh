#!/bin/bash
# Round 6, session p: 16-bit medians of 97-128 clients move to the bit-plane select (one lane per
# column pair): the defense tests, config 4's median at 128 clients as the bench reports it, its
# PMC traffic (two passes) and the SQ VALU table again.
set -o pipefail
OUT=gpurun_out/r06/p
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 420 python -u -m pytest tests/test_gpu_defense.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_defense.log 2>&1 || exit 1
B="--op median --config cfg4 --clients 128 --no-cpu-baseline"
timeout -k 10 240 python3 bench.py $B --steps 20 > $OUT/median_cfg4_k128.json 2> $OUT/median_cfg4_k128.err || exit 1
alg=$(python3 -c "import json; print(json.load(open('$OUT/median_cfg4_k128.json'))['roofline']['alg_bytes_per_step'])") || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o b \
  -- python3 bench.py $B --steps 3 --warmup 1 > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o b \
  -- python3 bench.py $B --steps 3 --warmup 1 > $OUT/write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py --fetch $OUT/fetch/b_counter_collection.csv --write $OUT/write/b_counter_collection.csv \
  --key "cfg4:single:median@K128" --kernel median_pk16_lanes_kernel --alg-bytes "$alg" --out $OUT/pmc_traffic_p.json || exit 1
timeout -k 10 900 python3 tools/median_valu.py collect > $OUT/median_valu_collect.log 2>&1 || exit 1
python3 tools/median_valu.py merge > $OUT/median_valu.json || exit 1
find $OUT gpurun_out/median_valu -name "*kernel_trace.csv" -size +1M -delete
tail -2 $OUT/pytest_defense.log; cat $OUT/pmc_traffic_p.json; python3 -c "import json; d=json.load(open('$OUT/median_cfg4_k128.json')); print(d['ms_per_step'], d['roofline'])"
