#!/bin/bash
# Round 4: the centred Gram on the bf16 matrix cores (three-way exact bf16
# split, six 16x16x32 MFMAs per 32 columns): distance-defense GPU tests, the
# A/B against the f32-MFMA kernel with each variant's error against the
# exact-difference kernel, and the Krum bench line.
set -o pipefail
O=gpurun_out/r04/k
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_defenses.py -x -q --timeout 120 --timeout-method thread \
    > $O/pytest.log 2>&1 \
 && GRAM_AB_DIR=tools/_abbuild timeout -k 10 300 python tools/gram_variants.py --rounds 9 --out $O/gram_variants.json \
    --variant "f32=-DFEDAGG_GRAM_SPLIT=0" --variant "fold1=-DFEDAGG_GRAM_SPLIT_FOLD=1" \
    --variant "fold8=-DFEDAGG_GRAM_SPLIT_FOLD=8" > $O/gram_variants.log 2>&1 \
 && timeout -k 10 300 python bench.py --op krum --steps 5 --warmup 2 --no-cpu-baseline > $O/krum_cfg3.json 2> $O/bench.err
rc=$?
tail -3 $O/pytest.log
cat $O/gram_variants.log | tail -6
python3 -c "import json; d=json.load(open('$O/krum_cfg3.json')); r=d['roofline']; print('krum', d['ms_per_step'], r['kernel_ms_per_step'], r['achieved'], r['frac'])" 2>/dev/null
exit $rc
