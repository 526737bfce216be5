#!/bin/bash
# Round 5: non-temporal stores in the small host-round pack (configs 1-2):
# the parity suites and the small-config agg() latency.
set -o pipefail
O=gpurun_out/r05/ad
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_simulation.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
 && timeout -k 10 300 python -u tools/small_agg_bench.py > $O/small_agg.txt 2>&1
rc=$?
tail -1 $O/pytest.log
tail -25 $O/small_agg.txt
exit $rc
