#!/bin/bash
# Round 5: bf16 chain at U1V8 from 256 clients.  New wide-tile tests first,
# then the whole GPU suite, the back-to-back A/B at config 4 and its bench
# line with rocprof stats.
set -o pipefail
O=gpurun_out/r05/n
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_large.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -u tools/ab_backtoback.py --dtype bf16 --K 512 --N 86567656 --variants shipped U1V4 U4V4_lowhalf --rounds 5 --launches 10 --out $O/ab_cfg4.json > $O/ab_cfg4.txt 2>&1 \
 && timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
grep -E "PASS|FAIL" $O/pytest_large.log | cut -c1-100
tail -1 $O/pytest_gpu.log
grep "^bf16" $O/ab_cfg4.txt
python3 -c "
import json; d=json.load(open('$O/bench_cfg4.json')); r=d['roofline']; print(round(d['ms_per_step'],4), r['kernel_ms_per_step'], r['achieved'], r['frac'], r['traffic'])"
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])" | head -2
exit $rc
