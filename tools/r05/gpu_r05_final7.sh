#!/bin/bash
# Round 5 closing check after the upload change (last code of the round): the whole GPU suite, smoke, the default bench line as
# the driver runs it, its rocprofv3 kernel stats, and the self-launched
# two-rank gloo rehearsal of the multi-GPU line (param + exchange + inprocess).
set -o pipefail
O=gpurun_out/r05/final7
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 \
 && timeout -k 10 420 python bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 > $O/gloo2_cfg3.json 2>> $O/bench.err
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -2 $O/pytest_gpu.log; tail -1 $O/smoke.log
python3 -c "
import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print(round(d['ms_per_step'],4), r['kernel_ms_per_step'], r['achieved'], r['frac'], d['cpu_baseline']['ms_per_aggregation'])" 2>/dev/null
exit $rc
