#!/bin/bash
# Round 3: the distance-defense kernels as they ship now (dist2's parallel
# finish, clip's clients in flight): parity tests, the clip A/B, bench lines
# and rocprofv3 kernel stats for --op krum / dist2 / clip at config 3, and
# FETCH_SIZE / WRITE_SIZE passes of dist2 and clip.
set -o pipefail
O=gpurun_out/r03/dist
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { echo "== $*" >&2; "$@"; }
B="python bench.py --no-cpu-baseline"
run timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_defenses.py -x -q --timeout 120 --timeout-method thread \
      > $O/test.log 2>&1 \
 && run timeout -k 10 300 python tools/robust_variants.py --rounds 10 > $O/clip_variants.txt 2>&1 \
 && run timeout -k 10 300 $B --op krum --steps 5 --warmup 1 > $O/bench_krum_cfg3.json 2> $O/bench.err \
 && run timeout -k 10 300 $B --op dist2 --steps 20 > $O/bench_dist2_cfg3.json 2>> $O/bench.err \
 && run timeout -k 10 300 $B --op clip --steps 20 > $O/bench_clip_cfg3.json 2>> $O/bench.err \
 && run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_krum -o krum \
      -- python3 bench.py --no-cpu-baseline --op krum --steps 5 --warmup 1 > $O/prof_krum.log 2>&1 \
 && run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dist2 -o dist2 \
      -- python3 bench.py --no-cpu-baseline --op dist2 --steps 20 > $O/prof_dist2.log 2>&1 \
 && run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_clip -o clip \
      -- python3 bench.py --no-cpu-baseline --op clip --steps 10 > $O/prof_clip.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch_dist2 -o dist2 \
      -- python3 bench.py --no-cpu-baseline --op dist2 --steps 3 --warmup 1 > $O/pmc_fetch_dist2.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch_clip -o clip \
      -- python3 bench.py --no-cpu-baseline --op clip --steps 3 --warmup 1 > $O/pmc_fetch_clip.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write_clip -o clip \
      -- python3 bench.py --no-cpu-baseline --op clip --steps 3 --warmup 1 > $O/pmc_write_clip.log 2>&1
rc=$?
tail -2 $O/test.log; cat $O/clip_variants.txt | grep clip; cat $O/bench_*.json | cut -c1-600
exit $rc
