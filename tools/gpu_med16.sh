#!/bin/bash
# Median kernels: the median GPU tests, then the 16-bit / many-client timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_defense.py -x -q --timeout 120 --timeout-method thread -k "median" > gpurun_out/med16_tests.log 2>&1 \
 && timeout -k 10 400 python -u tools/median_bench.py gpurun_out/median_bench_16.json --sixteen > gpurun_out/med16_bench.log 2>&1 \
 && timeout -k 10 400 python -u tools/median_bench.py gpurun_out/median_bench_all.json > gpurun_out/med_all_bench.log 2>&1
rc=$?
tail -3 gpurun_out/med16_tests.log; cat gpurun_out/med16_bench.log gpurun_out/med_all_bench.log
exit $rc
