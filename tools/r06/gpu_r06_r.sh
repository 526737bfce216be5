#!/bin/bash
# Round 6, session r: the whole GPU suite on the final library (column-kernel median for 129-1024
# clients, bit planes for 97-128), smoke, the default bench line with its rocprofv3 summary, and
# config 4 median line.
set -o pipefail
OUT=gpurun_out/r06/r
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err \
 && timeout -k 10 240 python bench.py --op median --config cfg4 --steps 10 --no-cpu-baseline > $OUT/median_cfg4.json 2> $OUT/median_cfg4.err \
 && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench \
      -- python3 bench.py --steps 25 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.log
rc=$?
find $OUT -name "*kernel_trace.csv" -size +1M -delete
tail -2 $OUT/pytest_gpu.log; cat $OUT/smoke.log; cat $OUT/bench.json
exit $rc
