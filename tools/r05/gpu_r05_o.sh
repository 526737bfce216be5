#!/bin/bash
# Round 5: fp32 tile shapes back to back at config 3's row (128 x 25,610,205)
# and config 5's (64 x 4,194,304).
set -o pipefail
O=gpurun_out/r05/o
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/ab_backtoback.py --dtype f32 --K 128 --N 25610205 --variants shipped U1V4 U2V4 U1V8 U4V2 U8V1 U2V2 --rounds 7 --launches 20 --out $O/ab_cfg3.json > $O/ab.txt 2>&1 \
 && timeout -k 10 300 python -u tools/ab_backtoback.py --dtype f32 --K 512 --N 25610205 --variants shipped U1V4 U2V4 U1V8 U4V2 --rounds 5 --launches 10 --out $O/ab_k512.json >> $O/ab.txt 2>&1
rc=$?
grep "^f32" $O/ab.txt
exit $rc
