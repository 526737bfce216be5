#!/bin/bash
# Round-end evidence: bench line, rocprofv3 kernel stats, two PMC passes.
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o bench \
      -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_${TAG} -o bench \
      -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_${TAG}.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_${TAG} -o bench \
      -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_${TAG}.log 2>&1
rc=$?
cat gpurun_out/bench_${TAG}.json
exit $rc
