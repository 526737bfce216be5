#!/bin/bash
# Round 5: the whole GPU suite after the MPI-order op, the alias programs, the
# non-finite Krum fallback and the fork-safe pack pool (rebuilt library).
set -o pipefail
O=gpurun_out/r05/b
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench.err
rc=$?
tail -3 $O/pytest_gpu.log; tail -1 $O/smoke.log
python3 -c "
import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print(round(d['ms_per_step'],4), r['kernel_ms_per_step'], r['achieved'], r['frac'])" 2>/dev/null
exit $rc
