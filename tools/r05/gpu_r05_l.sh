#!/bin/bash
# Round 5: back-to-back A/B of the bf16 tile shapes at config 4's shape.
set -o pipefail
O=gpurun_out/r05/l
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/ab_backtoback.py --dtype bf16 --K 512 --N 86567656 --variants shipped U4V4 U4V4_lowhalf U1V8 U2V4 --rounds 7 --launches 20 --out $O/ab_cfg4.json > $O/ab_cfg4.txt 2>&1 \
 && timeout -k 10 300 python -u tools/ab_backtoback.py --dtype bf16 --K 128 --N 86567656 --variants shipped U4V4 U4V4_lowhalf U2V4 --rounds 7 --launches 20 --out $O/ab_k128.json > $O/ab_k128.txt 2>&1
rc=$?
cat $O/ab_cfg4.txt $O/ab_k128.txt | grep "^bf16"
exit $rc
