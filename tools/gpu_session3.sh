#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest8.log 2>&1 \
 && timeout -k 10 300 python tools/tune_wsum.py --rounds 6 > gpurun_out/tune4.log 2>&1 \
 && for c in cfg1 cfg2 cfg5 cfg3; do timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_$c.json 2>gpurun_out/bench_$c.err || exit 1; done
rc=$?
tail -2 gpurun_out/pytest8.log; grep -E "U4V4nt |U8V4nt |copy" gpurun_out/tune4.log
for c in cfg1 cfg2 cfg5 cfg3; do python -c "import json,sys; d=json.load(open('gpurun_out/bench_$c.json')); print('$c', 'ms/step %.4f'%d['ms_per_step'], 'kernel ms %.4f'%d['roofline']['kernel_ms_per_step'], 'GB/s', d['roofline']['achieved'])" 2>/dev/null; done
exit $rc
