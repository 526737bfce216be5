#!/bin/bash
# Round 5: every bench line of DESIGN §5's "other configs and ops" table,
# re-measured after the reduce_into issue-time change (one box session)
# (no rocprof in this pass).
set -o pipefail
O=gpurun_out/r05/aj
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
run() {  # name, args...
  local n=$1; shift
  [ $ok = 0 ] || return
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$n.json 2>> $O/bench.err || { ok=1; echo "FAILED $n"; }
}
run cfg1 --config cfg1
run cfg2 --config cfg2
run cfg3 --config cfg3
run cfg4 --config cfg4
run cfg4_acc32 --config cfg4 --acc fp32
run cfg5_sgd --config cfg5 --fedopt sgd
run cfg5_adam --config cfg5 --fedopt adam
run median_cfg3 --op median --config cfg3
run median_cfg4 --op median --config cfg4
run krum_cfg3 --op krum --config cfg3
run dist2_cfg3 --op dist2 --config cfg3
run clip_cfg3 --op clip --config cfg3
run rlr_cfg3 --op rlr --config cfg3
run mpi_cfg3 --op mpi --config cfg3
run secagg --op secagg --config cfg3
run lsa --op lsa --config cfg3
python3 - <<PY
import json, glob, os
for f in sorted(glob.glob("$O/*.json")):
    try:
        d = json.load(open(f)); r = d["roofline"]
        print(f"{os.path.basename(f)[:-5]:12s} {d['ms_per_step']:9.4f} ms  {r['achieved']:8.1f} {r['unit']}  frac {r['frac']}")
    except Exception as e:
        print(f, "unreadable", e)
PY
exit $ok
