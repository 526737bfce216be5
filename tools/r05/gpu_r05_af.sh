#!/bin/bash
# Round 5: the ingest's layout check on lists, dict update for the rebinding.
set -o pipefail
O=gpurun_out/r05/af
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_cross_silo.py tests/test_gpu_host_copy.py tests/test_gpu_multidev.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
 && timeout -k 10 200 python -u tools/profile_arrival.py --config cfg5 > $O/prof_arrival_cfg5.txt 2>&1 \
 && timeout -k 10 300 python -u tools/e2e_configs.py --config cfg5 --rounds 6 --out $O/e2e_cfg5.json > $O/e2e_cfg5.log 2>&1
rc=$?
tail -1 $O/pytest.log
head -12 $O/prof_arrival_cfg5.txt | tail -6
python3 -c "
import json; d=json.load(open('$O/e2e_cfg5.json')); x=d['xsilo']
print([r['arrival_ms_median'] for r in x['rounds']], x['ingest_GBps_median'], d['agg_call'])"
exit $rc
