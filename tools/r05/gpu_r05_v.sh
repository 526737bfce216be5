#!/bin/bash
# Round 5 experiment: persistent streaming / staggered tiles against the
# shipped fp32 tiles at config 3 (and K = 512), back to back.
set -o pipefail
O=gpurun_out/r05/v
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/ab_backtoback.py --table f32 --dtype f32 --K 128 --N 25610205 --variants shipped U4V4nt S_V4D4_c4 S_V4D3_c4 S_V2D6_c4 S_V4D2_c4 S_V2D4_c6 T_U4_c4 T_U4_c4_flat T_U4_c3 T_U2_c4 U4V4nt_p4 --rounds 7 --launches 20 --out $O/ab_cfg3.json > $O/ab.txt 2>&1 \
 && timeout -k 10 300 python -u tools/ab_backtoback.py --table f32 --dtype f32 --K 512 --N 25610205 --variants shipped T_U4_c3 T_U4_c4_flat S_V4D4_c4 --rounds 5 --launches 10 --out $O/ab_k512.json >> $O/ab.txt 2>&1
rc=$?
grep "^f32" $O/ab.txt
exit $rc
