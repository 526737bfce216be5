#!/bin/bash
# Round 3: narrow-pack policy -- GPU suite, many-client probes, tiny re-sweep.
set -o pipefail
O=gpurun_out/r03/narrow1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { echo "== $*" >&2; "$@"; }
run timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -2 $O/test.log
for d in bf16 f16 f32; do
  run timeout -k 10 200 python tools/manyclient_probe.py --dtype $d --out r03/narrow1/manyclient_$d > $O/manyclient_$d.log 2>&1 \
    || { tail $O/manyclient_$d.log; exit 1; }
done
grep -h reference $O/manyclient_*.log
run timeout -k 10 400 python tools/tune_tiny.py --rounds 9 --out $O/tune_tiny.json > $O/tune_tiny.txt 2>&1 || { tail $O/tune_tiny.txt; exit 1; }
cut -c1-90 $O/tune_tiny.txt
