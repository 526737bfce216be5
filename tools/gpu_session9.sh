#!/bin/bash
# Pipelined device-dict path: GPU tests, then the config-3 agg() timing.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r01f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 \
 && timeout -k 10 300 python tools/devdict_bench.py --reps 7 > gpurun_out/devdict_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_${TAG}.log; tail -20 gpurun_out/devdict_${TAG}.log
exit $rc
