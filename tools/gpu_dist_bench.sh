#!/bin/bash
# Distance-defense kernels on the GPU box: bench lines for --op krum / dist2 /
# clip at config 3 (and krum at configs 2 and 5), rocprofv3 kernel stats of
# the krum and clip runs, FETCH_SIZE / WRITE_SIZE passes of dist2 and clip.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
TAG=${1:-r02d}
O=gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { echo "== $*" >&2; "$@"; }
B="python bench.py --no-cpu-baseline"
run timeout -k 10 300 $B --op krum --steps 5 --warmup 1 > $O/bench_krum_cfg3.json 2> $O/bench.err \
 && run timeout -k 10 300 $B --op dist2 --steps 20 > $O/bench_dist2_cfg3.json 2>> $O/bench.err \
 && run timeout -k 10 300 $B --op clip --steps 20 > $O/bench_clip_cfg3.json 2>> $O/bench.err \
 && run timeout -k 10 300 $B --op krum --config cfg2 --steps 20 > $O/bench_krum_cfg2.json 2>> $O/bench.err \
 && run timeout -k 10 300 $B --op krum --config cfg5 --steps 20 > $O/bench_krum_cfg5.json 2>> $O/bench.err \
 && run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_krum -o bench \
      -- python3 bench.py --no-cpu-baseline --op krum --steps 5 --warmup 1 > $O/prof_krum.log 2>&1 \
 && run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_clip -o bench \
      -- python3 bench.py --no-cpu-baseline --op clip --steps 10 > $O/prof_clip.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch_dist2 -o bench \
      -- python3 bench.py --no-cpu-baseline --op dist2 --steps 3 --warmup 1 > $O/pmc_fetch_dist2.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch_clip -o bench \
      -- python3 bench.py --no-cpu-baseline --op clip --steps 3 --warmup 1 > $O/pmc_fetch_clip.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write_clip -o bench \
      -- python3 bench.py --no-cpu-baseline --op clip --steps 3 --warmup 1 > $O/pmc_write_clip.log 2>&1
rc=$?
cat $O/bench_*.json
exit $rc
