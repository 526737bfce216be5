#!/bin/bash
# Round 5: to_host in one piece against 16 MB pieces, config 3, same box.
set -o pipefail
O=gpurun_out/r05/ai
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
FEDAGG_TO_HOST_CHUNK=0 timeout -k 10 500 python -u tools/e2e_configs.py --config cfg3 --rounds 6 --out $O/e2e_cfg3_one.json > $O/one.log 2>&1 \
 && timeout -k 10 500 python -u tools/e2e_configs.py --config cfg3 --rounds 6 --out $O/e2e_cfg3_chunked.json > $O/chunked.log 2>&1 \
 && FEDAGG_TO_HOST_CHUNK=0 timeout -k 10 500 python -u tools/e2e_configs.py --config cfg3 --rounds 6 --out $O/e2e_cfg3_one_b.json > $O/one_b.log 2>&1
rc=$?
for f in one chunked one_b; do python3 -c "
import json; d=json.load(open('$O/e2e_cfg3_$f.json')); x=d['xsilo']
print('$f', [r['broadcast_to_host_ms'] for r in x['rounds']], x['round_end_to_host_ms_median'], x['ingest_GBps_median'])
" 2>/dev/null; done
exit $rc
