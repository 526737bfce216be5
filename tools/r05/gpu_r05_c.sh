#!/bin/bash
# Round 5: host-resident rounds end to end for configs 5 and 4 (cross-silo
# mirror + the agg() call shape), and the G = 4 ingest A/B with one shared
# copy stream (is the +13 % the one PCIe link, or the per-shard streams?).
set -o pipefail
O=gpurun_out/r05/c
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/e2e_configs.py --config cfg5 --out $O/e2e_cfg5.json > $O/e2e_cfg5.log 2>&1 \
 && timeout -k 10 420 python tools/e2e_configs.py --config cfg4 --rounds 2 --agg-reps 2 --out $O/e2e_cfg4.json > $O/e2e_cfg4.log 2>&1 \
 && timeout -k 10 420 python tools/multidev_bench.py --clients 32 --reps 3 --shards 1 2 4 --ingest --shared-copy --out $O/multidev_ingest.json > $O/multidev.log 2>&1
rc=$?
tail -2 $O/e2e_cfg5.log; tail -2 $O/e2e_cfg4.log; grep ingest $O/multidev.log
python3 - <<'PY'
import json
for c in ("cfg5", "cfg4"):
    try:
        d = json.load(open(f"gpurun_out/r05/c/e2e_{c}.json"))
        print(c, d["link"], d["xsilo"]["ingest_GBps_median"], d["xsilo"]["round_end_ms_median"], d["agg_call"])
    except Exception as e:
        print(c, "missing", e)
PY
exit $rc
