#!/bin/bash
# Round 4, closing check after the last Gram changes: the GPU suite, smoke,
# the default bench line (as the driver runs it) and the Krum line.
set -o pipefail
O=gpurun_out/r04/final4
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench.err \
 && timeout -k 10 300 python bench.py --op krum --steps 10 --warmup 3 > $O/krum_cfg3.json 2>> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_krum -o run \
      -- python3 bench.py --op krum --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_krum.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -1 $O/pytest_gpu.log; tail -1 $O/smoke.log
for f in $O/bench_default.json $O/krum_cfg3.json; do python3 -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('$f'.split('/')[-1], round(d['ms_per_step'],4), r['kernel_ms_per_step'], r['achieved'], r['frac'], (d['cpu_baseline'] or {}).get('ms_per_aggregation'))"; done
exit $rc
