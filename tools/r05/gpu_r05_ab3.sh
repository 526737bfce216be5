#!/bin/bash
# Round 5: non-temporal host pack; the e2e
# rounds of configs 3 and 5 with the by-buffer broadcast copy beside the
# per-key one.
set -o pipefail
O=gpurun_out/r05/ab3
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_copy.py tests/test_gpu_cross_silo.py tests/test_cross_silo.py -m "gpu or not gpu" -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
 && timeout -k 10 500 python -u tools/e2e_configs.py --config cfg3 --rounds 6 --out $O/e2e_cfg3.json > $O/e2e_cfg3.log 2>&1 \
 && timeout -k 10 300 python -u tools/e2e_configs.py --config cfg5 --rounds 6 --out $O/e2e_cfg5.json > $O/e2e_cfg5.log 2>&1
rc=$?
tail -2 $O/pytest.log
for c in cfg3 cfg5; do python3 -c "
import json; d=json.load(open('$O/e2e_$c.json')); x=d['xsilo']
for r in x['rounds']: print('$c', r['aggregate_ms'], r['broadcast_d2h_ms'], r['broadcast_to_host_ms'], r['round_end_ms'], r['round_end_to_host_ms'], r['ingest_GBps'])
" 2>/dev/null; done
exit $rc
