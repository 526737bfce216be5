#!/bin/bash
# Round 5: repeat the lines of r05/y that moved against earlier rounds
# (clip, config 5 SGD / Adam, config 4 acc fp32), three times each, in one box
# session.
set -o pipefail
O=gpurun_out/r05/z
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
for i in 1 2 3; do
  for spec in "clip --op clip --config cfg3" "cfg5_sgd --config cfg5 --fedopt sgd" "cfg5_adam --config cfg5 --fedopt adam" "cfg4_acc32 --config cfg4 --acc fp32" "cfg4 --config cfg4"; do
    set -- $spec; n=$1; shift
    [ $ok = 0 ] || break
    timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/${n}_$i.json 2>> $O/bench.err || { ok=1; echo "FAILED $n"; }
  done
done
python3 - <<PY
import json, glob, os
for f in sorted(glob.glob("$O/*.json")):
    d = json.load(open(f)); r = d["roofline"]
    print(f"{os.path.basename(f)[:-5]:14s} {d['ms_per_step']:9.4f} ms  kernel {r['kernel_ms_per_step']}  frac {r['frac']}")
PY
exit $ok
