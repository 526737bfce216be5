#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest10.log 2>&1 \
 && timeout -k 10 300 python bench.py --config cfg4 --steps 20 --no-cpu-baseline > gpurun_out/bench_cfg4_ref.json 2>gpurun_out/b4.err \
 && timeout -k 10 300 python bench.py --config cfg4 --acc fp32 --steps 20 --no-cpu-baseline > gpurun_out/bench_cfg4_fp32.json 2>>gpurun_out/b4.err \
 && timeout -k 10 300 python bench.py --config cfg5 --fedopt --steps 100 --no-cpu-baseline > gpurun_out/bench_cfg5_fedopt.json 2>gpurun_out/b5.err \
 && timeout -k 10 300 python bench.py --config cfg5 --steps 100 --no-cpu-baseline > gpurun_out/bench_cfg5.json 2>gpurun_out/b5.err \
 && timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline > gpurun_out/bench_cfg3.json 2>gpurun_out/b3.err
rc=$?
tail -2 gpurun_out/pytest10.log
for f in bench_cfg4_ref bench_cfg4_fp32 bench_cfg5_fedopt bench_cfg5 bench_cfg3; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['n_gpus'], 'ms/step %.4f'%d['ms_per_step'], 'kernel ms %.4f'%d['roofline']['kernel_ms_per_step'], 'GB/s', d['roofline']['achieved'], '%.4g'%d['value'])" 2>&1 | tail -1; done
exit $rc
