#!/bin/bash
# Round 3, end of session: GPU suite, smoke, headline bench + rocprofv3 kernel
# stats, and the defense bench lines DESIGN quotes.  Each GPU step under its own
# time limit; the chain stops at the first failure.
set -o pipefail
O=gpurun_out/r03_final
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench \
      -- python3 bench.py --steps 20 --no-cpu-baseline > $O/prof.log 2>&1 \
 && timeout -k 10 300 python bench.py --op median --config cfg4 --clients 512 --steps 5 --warmup 2 --no-cpu-baseline > $O/median_cfg4_k512.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --op median --steps 10 --warmup 2 --no-cpu-baseline > $O/median_cfg3.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --op krum --steps 5 --warmup 2 --no-cpu-baseline > $O/krum_cfg3.json 2>> $O/bench.err
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -3 $O/pytest_gpu.log; cat $O/smoke.log 2>/dev/null; cat $O/bench.json 2>/dev/null
for f in median_cfg4_k512 median_cfg3 krum_cfg3; do python3 -c "import json,sys; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r.get('valu', {}).get('frac'))" 2>/dev/null; done
exit $rc
