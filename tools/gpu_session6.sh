#!/bin/bash
# GPU tests, then config-5 FedOpt / FedAvg benches and the headline bench.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r01d}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 \
 && timeout -k 10 300 python bench.py --config cfg5 --fedopt sgd --steps 100 --no-cpu-baseline > gpurun_out/bench_cfg5_sgd_${TAG}.json 2>gpurun_out/b5.err \
 && timeout -k 10 300 python bench.py --config cfg5 --fedopt adam --steps 100 --no-cpu-baseline > gpurun_out/bench_cfg5_adam_${TAG}.json 2>>gpurun_out/b5.err \
 && timeout -k 10 300 python bench.py --config cfg5 --steps 100 --no-cpu-baseline > gpurun_out/bench_cfg5_${TAG}.json 2>>gpurun_out/b5.err \
 && timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline > gpurun_out/bench_cfg3_${TAG}.json 2>gpurun_out/b3.err
rc=$?
tail -2 gpurun_out/pytest_${TAG}.log
for f in bench_cfg5_sgd bench_cfg5_adam bench_cfg5 bench_cfg3; do python -c "import json; d=json.load(open('gpurun_out/${f}_${TAG}.json')); print('$f', 'ms/step %.4f'%d['ms_per_step'], 'kernel ms %.4f'%d['roofline']['kernel_ms_per_step'], 'GB/s', d['roofline']['achieved'])" 2>&1 | tail -1; done
exit $rc
