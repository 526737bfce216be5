#!/bin/bash
# Round 5 follow-up: the MPI muldiv kernel's every-tile parity, the simulation
# and parity suites, and the kernel's own bench line (--op mpi) with its
# rocprofv3 kernel stats.
set -o pipefail
O=gpurun_out/r05/g
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_simulation.py tests/test_gpu_parity.py tests/test_gpu_cross_silo.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python bench.py --op mpi --no-cpu-baseline > $O/bench_mpi.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 bench.py --op mpi --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -2 $O/pytest_gpu.log
cat $O/bench_mpi.json
exit $rc
