#!/bin/bash
# Round 5: tile shapes of the bf16 fp32-accumulated chain (acc_mode fp32).
set -o pipefail
O=gpurun_out/r05/t
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
for KN in "512 86567656" "128 86567656" "512 21641914" "512 43283828" "64 86567656"; do
  set -- $KN
  timeout -k 10 200 python -u tools/ab_backtoback.py --dtype bf16acc32 --K $1 --N $2 --variants shipped U1V8 U1V4 U2V4 --rounds 5 --launches 10 >> $O/ab.txt 2>&1 || { ok=1; break; }
done
grep "^bf16" $O/ab.txt
exit $ok
