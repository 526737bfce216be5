#!/bin/bash
# Round 5: U1V8 against the shipped U1V4 for the bf16 chain by client count.
set -o pipefail
O=gpurun_out/r05/m
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
for KN in "128 86567656" "192 86567656" "256 86567656" "384 86567656" "256 16777216" "512 16777216" "512 8388608" "1024 8388608"; do
  set -- $KN
  timeout -k 10 200 python -u tools/ab_backtoback.py --dtype bf16 --K $1 --N $2 --variants shipped U1V8 U2V4 --rounds 5 --launches 10 --out $O/ab_K$1_N$2.json >> $O/ab.txt 2>&1 || { ok=1; break; }
done
grep "^bf16" $O/ab.txt
exit $ok
