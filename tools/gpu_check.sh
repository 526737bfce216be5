#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread> gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
 && timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o bench \
      -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log; cat gpurun_out/smoke_${TAG}.log 2>/dev/null; cat gpurun_out/bench_${TAG}.json 2>/dev/null
exit $rc
