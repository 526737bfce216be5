#!/bin/bash
# Round 5: fused SGD at the 128-VGPR cap.  Whole GPU suite and the config 5
# SGD / Adam bench lines.
set -o pipefail
O=gpurun_out/r05/aa
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python bench.py --config cfg5 --fedopt sgd --no-cpu-baseline > $O/cfg5_sgd.json 2> $O/bench.err \
 && timeout -k 10 300 python bench.py --config cfg5 --fedopt adam --no-cpu-baseline > $O/cfg5_adam.json 2>> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 bench.py --config cfg5 --fedopt sgd --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -1 $O/pytest_gpu.log
for f in $O/cfg5_sgd.json $O/cfg5_adam.json; do python3 -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('$f', round(d['ms_per_step'],4), r['kernel_ms_per_step'], r['achieved'], r['frac'])"; done
exit $rc
