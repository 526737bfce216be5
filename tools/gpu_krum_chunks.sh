#!/bin/bash
# After the line-aligned chunk tables: the GPU suite's defense tests, the
# Krum / dist2 bench lines and rocprofv3 kernel stats for Krum.
set -o pipefail
O=gpurun_out/r03/krum_chunks
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python bench.py --op krum --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_krum.json 2>/dev/null \
 && timeout -k 10 300 python bench.py --op dist2 --steps 20 --warmup 2 --no-cpu-baseline > $O/bench_dist2.json 2>/dev/null \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_krum -o b \
      -- python3 bench.py --op krum --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_krum.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -1 $O/pytest_gpu.log
for f in krum dist2; do python3 -c "import json; d=json.load(open('$O/bench_$f.json')); print('$f', d['ms_per_step'], d['roofline'])" 2>/dev/null; done
grep -h "pairgram\|finish" $O/prof_krum/b_kernel_stats.csv 2>/dev/null | cut -c1-160
exit $rc
