#!/bin/bash
# Round 4: Krum's centred Gram with A-fragment reuse (A/B in one process,
# bit-identical outputs required), and the in-process multi-device ingest
# with concurrent per-shard packs (tools/multidev_bench.py, G = 1 / 2 / 4
# shards on the box's one GPU) after its GPU tests.
set -o pipefail
O=gpurun_out/r04/d
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GRAM_AB_DIR=tools/_abbuild timeout -k 10 300 python tools/gram_variants.py --rounds 9 --out $O/gram_variants.json \
    --variant "reuse=-DFEDAGG_GRAM_AREUSE=1" --variant "base=-DFEDAGG_GRAM_AREUSE=0" > $O/gram_variants.log 2>&1 \
 && timeout -k 10 300 python -u -m pytest tests/test_gpu_multidev.py tests/test_gpu_dist_defenses.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1 \
 && timeout -k 10 400 python tools/multidev_bench.py --clients 32 --reps 3 --out $O/multidev_bench.json > $O/multidev_bench.log 2>&1 \
 && timeout -k 10 300 python bench.py --op krum --steps 5 --warmup 2 --no-cpu-baseline > $O/krum_cfg3.json 2> $O/bench.err
rc=$?
cat $O/gram_variants.log | tail -4
tail -3 $O/pytest.log
cat $O/multidev_bench.json
python3 -c "import json; d=json.load(open('$O/krum_cfg3.json')); r=d['roofline']; print('krum', d['ms_per_step'], r['kernel_ms_per_step'], r['achieved'], r['frac'])" 2>/dev/null
exit $rc
