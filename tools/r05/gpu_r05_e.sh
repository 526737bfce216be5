#!/bin/bash
# Round 5: the resident-bucket round end (cross-silo aggregate() reduces the
# ingested rows directly): its GPU tests, then the end-to-end rounds again.
set -o pipefail
O=gpurun_out/r05/e
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_cross_silo.py tests/test_gpu_multidev.py tests/test_gpu_round_end.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
 && timeout -k 10 300 python tools/e2e_configs.py --config cfg5 --out $O/e2e_cfg5.json > $O/e2e_cfg5.log 2>&1 \
 && timeout -k 10 300 python tools/e2e_configs.py --config cfg3 --rounds 3 --agg-reps 2 --out $O/e2e_cfg3.json > $O/e2e_cfg3.log 2>&1 \
 && timeout -k 10 420 python tools/e2e_configs.py --config cfg4 --rounds 2 --agg-reps 1 --out $O/e2e_cfg4.json > $O/e2e_cfg4.log 2>&1
rc=$?
tail -2 $O/pytest.log
python3 - <<'PY'
import json
for c in ("cfg5", "cfg3", "cfg4"):
    try:
        d = json.load(open(f"gpurun_out/r05/e/e2e_{c}.json"))
        print(c, d["xsilo"]["ingest_GBps_median"], d["xsilo"]["round_end_ms_median"], [(x["aggregate_ms"], x["broadcast_d2h_ms"]) for x in d["xsilo"]["rounds"]], d["agg_call"]["s_median"])
    except Exception as e:
        print(c, "missing", e)
PY
exit $rc
