#!/bin/bash
# Round 6, session c: the whole GPU suite on the round-6 library (OptRepo epilogues, device round,
# folded knobs, tuning entries gated out), smoke, the default bench line and its rocprofv3 summary.
set -o pipefail
OUT=gpurun_out/r06/c
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err \
 && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench \
      -- python3 bench.py --steps 25 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.log
rc=$?
tail -3 $OUT/pytest_gpu.log; cat $OUT/smoke.log 2>/dev/null; cat $OUT/bench.json 2>/dev/null
exit $rc
