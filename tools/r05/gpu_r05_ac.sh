#!/bin/bash
# Round 5: fp32 FedAvg time against client count at config 3's row length
# (intercept and per-client slope of the shipped tiles).
set -o pipefail
O=gpurun_out/r05/ac
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
for K in 1 2 4 8 16 32 64 128 192 256 384 512; do
  timeout -k 10 200 python -u tools/ab_backtoback.py --table f32 --dtype f32 --K $K --N 25610205 --variants shipped --rounds 5 --launches 20 >> $O/ab.txt 2>&1 || { ok=1; break; }
done
grep "^f32" $O/ab.txt
exit $ok
