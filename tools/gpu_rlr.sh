#!/bin/bash
# Robust-learning-rate defense: its GPU tests, then a timing at config 3.
set -o pipefail
mkdir -p gpurun_out/rlr
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_defenses.py -x -q --timeout 300 --timeout-method thread -k "robust_learning_rate" > gpurun_out/rlr/tests.log 2>&1 \
 && timeout -k 10 300 python bench.py --op rlr --steps 20 --no-cpu-baseline > gpurun_out/rlr/bench_rlr_cfg3.json 2> gpurun_out/rlr/bench.err
rc=$?
tail -3 gpurun_out/rlr/tests.log; cat gpurun_out/rlr/bench_rlr_cfg3.json
exit $rc
