#!/bin/bash
# Round 5: keys past the 32-bit element / byte ranges (tests/test_gpu_large.py).
set -o pipefail
O=gpurun_out/r05/h
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_large.log 2>&1
rc=$?
tail -15 $O/pytest_large.log
exit $rc
