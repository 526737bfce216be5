#!/bin/bash
# Round 5: bf16 reference chain shipped at U1V4 tiles.  Whole GPU suite, the
# config 4 bench line with rocprof stats, PMC traffic of the same line.
set -o pipefail
O=gpurun_out/r05/k
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -1 $O/pytest_gpu.log
python3 -c "
import json; d=json.load(open('$O/bench_cfg4.json')); r=d['roofline']; print(round(d['ms_per_step'],4), r['kernel_ms_per_step'], r['achieved'], r['frac'], r['traffic'])"
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])" | head -2
exit $rc
