#!/bin/bash
# Round-2 evidence on the GPU box: the headline bench line and its rocprofv3
# kernel stats, the median and the new fused server steps through bench.py,
# and FETCH_SIZE / WRITE_SIZE passes (separate runs) for the median kernels
# that changed this round.  Every GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { echo "== $*" >&2; "$@"; }
run timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err \
 && run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench \
      -- python3 bench.py --steps 20 --no-cpu-baseline > $O/prof_bench.log 2>&1 \
 && run timeout -k 10 300 python bench.py --op median --steps 20 --no-cpu-baseline > $O/bench_median_cfg3.json 2>> $O/bench.err \
 && run timeout -k 10 300 python bench.py --op median --config cfg4 --steps 20 --no-cpu-baseline > $O/bench_median_cfg4.json 2>> $O/bench.err \
 && run timeout -k 10 300 python bench.py --config cfg5 --fedopt rmsprop --steps 50 --no-cpu-baseline > $O/bench_cfg5_rmsprop.json 2>> $O/bench.err \
 && run timeout -k 10 300 python bench.py --config cfg5 --fedopt adamw --steps 50 --no-cpu-baseline > $O/bench_cfg5_adamw.json 2>> $O/bench.err \
 && run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_median -o bench \
      -- python3 bench.py --op median --steps 20 --no-cpu-baseline > $O/prof_median.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch_median3 -o bench \
      -- python3 bench.py --op median --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch_median3.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write_median3 -o bench \
      -- python3 bench.py --op median --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write_median3.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch_median4 -o bench \
      -- python3 bench.py --op median --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch_median4.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write_median4 -o bench \
      -- python3 bench.py --op median --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write_median4.log 2>&1
rc=$?
cat $O/bench.json
exit $rc
