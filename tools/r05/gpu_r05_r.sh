#!/bin/bash
# Round 5: is the fp32 headline losing time to the last partial round of
# workgroups?  Per-byte rate of the shipped U4V4 tiles at row lengths that
# give whole and fractional numbers of resident rounds (1,024 workgroups of
# 4,096 elements resident at once).
set -o pipefail
O=gpurun_out/r05/r
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
for N in 25165824 25610205 26214400 27262976 29360128 20971520 23068672; do
  timeout -k 10 200 python -u tools/ab_backtoback.py --dtype f32 --K 128 --N $N --variants shipped U1V4 --rounds 5 --launches 20 >> $O/ab.txt 2>&1 || { ok=1; break; }
done
grep "^f32" $O/ab.txt
exit $ok
