#!/bin/bash
# Median GPU tests with the current library, then the SQ passes for
# profiles/median_valu.json and the median bench lines that read it.
set -o pipefail
O=gpurun_out/median_valu
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "median or defense or config" --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python tools/median_valu.py collect > $O/collect.log 2>&1 || { tail -20 $O/collect.log; exit 1; }
python tools/median_valu.py merge || exit 1
for a in "--config cfg3" "--config cfg4" "--config cfg4 --clients 512" "--config cfg3 --clients 512"; do
  timeout -k 10 300 python bench.py --op median $a --steps 5 --warmup 2 --no-cpu-baseline >> $O/bench.jsonl 2>> $O/bench.err || exit 1
done
cat $O/bench.jsonl
