#!/bin/bash
# Round 4: the split-bf16 Gram as shipped (4-wave kernel): distance-defense GPU
# tests, the A/B against the f32 kernel and the two experimental variants, the
# Krum bench line and its rocprofv3 kernel stats.
set -o pipefail
O=gpurun_out/r04/y
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_defenses.py tests/test_gpu_defense.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1 \
 && GRAM_AB_DIR=tools/_abbuild timeout -k 10 300 python tools/gram_variants.py --rounds 9 --out $O/gram_variants.json \
    --variant "f32=-DFEDAGG_GRAM_SPLIT=0" --variant "split2=-DFEDAGG_GRAM_SPLIT=2" \
    --variant "ws4=-DFEDAGG_GRAM_SPLIT=3,-DFEDAGG_GRAM_WS_PD=4" > $O/gram_variants.log 2>&1 \
 && timeout -k 10 300 python bench.py --op krum --steps 10 --warmup 3 > $O/krum_cfg3.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 bench.py --op krum --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -2 $O/pytest.log
grep -v amdgpu.ids $O/gram_variants.log | tail -5
python3 -c "import json; d=json.load(open('$O/krum_cfg3.json')); r=d['roofline']; print('krum', d['ms_per_step'], r['kernel_ms_per_step'], r['achieved'], r['frac'], r.get('useful_tflops'), d['cpu_baseline'])" 2>/dev/null
exit $rc
