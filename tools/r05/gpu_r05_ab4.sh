#!/bin/bash
# Round 5: config 4's end-to-end rounds on the final code (to_host beside the
# per-key copy; the non-temporal pack).
set -o pipefail
O=gpurun_out/r05/ab4
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u tools/e2e_configs.py --config cfg4 --rounds 4 --out $O/e2e_cfg4.json > $O/e2e_cfg4.log 2>&1
rc=$?
python3 -c "
import json; d=json.load(open('$O/e2e_cfg4.json')); x=d['xsilo']
for r in x['rounds']: print(r)
print(d['agg_call'])"
exit $rc
