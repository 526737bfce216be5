#!/bin/bash
# Round 4: Krum Gram variants (fp64 fold interval, straight-line tiles) and
# compute-only diagnostics, one process.
set -o pipefail
O=gpurun_out/r04/f
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GRAM_AB_DIR=tools/_abbuild timeout -k 10 400 python tools/gram_variants.py --rounds 9 --out $O/gram_map.json \
    --variant "map0=-DFEDAGG_GRAM_MAP=0" --variant "map0f4=-DFEDAGG_GRAM_MAP=0,-DFEDAGG_GRAM_FOLD=4" --variant "map1f2=-DFEDAGG_GRAM_FOLD=2" \
    --variant "map1f4=-DFEDAGG_GRAM_FOLD=4" --variant "map1st=-DFEDAGG_GRAM_STRAIGHT=1" \
    --variant "map1nostage=-DFEDAGG_GRAM_DIAG=2" \
    > $O/gram_variants.log 2>&1 \
 && timeout -k 10 600 python tools/multidev_bench.py --clients 32 --reps 4 --ab-pack --out $O/multidev_ab.json > $O/multidev_ab.log 2>&1
rc=$?
grep ms $O/gram_variants.log
grep "host\|device" $O/multidev_ab.log
python3 -c "import json; print(json.load(open('$O/multidev_ab.json')).get('host_spawn_ms'))"
exit $rc
