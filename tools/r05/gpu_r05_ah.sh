#!/bin/bash
# Round 5: to_host with the chunked D2H and the overlapped scatter.
set -o pipefail
O=gpurun_out/r05/ah
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_copy.py tests/test_gpu_cross_silo.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
 && timeout -k 10 500 python -u tools/e2e_configs.py --config cfg3 --rounds 6 --out $O/e2e_cfg3.json > $O/e2e_cfg3.log 2>&1 \
 && timeout -k 10 300 python -u tools/e2e_configs.py --config cfg5 --rounds 6 --out $O/e2e_cfg5.json > $O/e2e_cfg5.log 2>&1
rc=$?
tail -1 $O/pytest.log
for c in cfg3 cfg5; do python3 -c "
import json; d=json.load(open('$O/e2e_$c.json')); x=d['xsilo']
print('$c', [r['broadcast_d2h_ms'] for r in x['rounds']], [r['broadcast_to_host_ms'] for r in x['rounds']], x['round_end_to_host_ms_median'], x['ingest_GBps_median'])
" 2>/dev/null; done
exit $rc
