#!/bin/bash
# Round 4: the 8-wave split Gram (FEDAGG_GRAM_SPLIT=2) as the shipped kernel:
# distance-defense GPU tests, A/B against the 4-wave kernel and f32, bench line.
set -o pipefail
O=gpurun_out/r04/z
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_defenses.py tests/test_gpu_defense.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1 \
 && GRAM_AB_DIR=tools/_abbuild timeout -k 10 300 python tools/gram_variants.py --rounds 11 --out $O/gram_variants.json \
    --variant "split1=-DFEDAGG_GRAM_SPLIT=1" --variant "f32=-DFEDAGG_GRAM_SPLIT=0" > $O/gram_variants.log 2>&1 \
 && timeout -k 10 300 python bench.py --op krum --steps 10 --warmup 3 > $O/krum_cfg3.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 bench.py --op krum --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -2 $O/pytest.log
grep -v amdgpu.ids $O/gram_variants.log | tail -4
python3 -c "import json; d=json.load(open('$O/krum_cfg3.json')); r=d['roofline']; print('krum', d['ms_per_step'], r['kernel_ms_per_step'], r['achieved'], r['frac'], r.get('useful_tflops'))" 2>/dev/null
exit $rc
