#!/bin/bash
# Round 5: tile shapes of the bf16 -> fp32 partial (client-axis config 4: 128
# of the 512 clients per GPU) and of the bf16 chain at 4-GPU-shard sizes.
set -o pipefail
O=gpurun_out/r05/p
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/ab_backtoback.py --dtype bf16f32 --K 128 --N 86567656 --variants shipped U1V4 U2V4 U1V8 U4V2 U2V2 U8V1 --rounds 7 --launches 10 --out $O/ab_f32out_k128.json > $O/ab.txt 2>&1 \
 && timeout -k 10 300 python -u tools/ab_backtoback.py --dtype bf16f32 --K 64 --N 86567656 --variants shipped U1V4 U2V4 U1V8 U4V2 --rounds 7 --launches 10 --out $O/ab_f32out_k64.json >> $O/ab.txt 2>&1 \
 && timeout -k 10 300 python -u tools/ab_backtoback.py --dtype bf16 --K 512 --N 21641914 --variants shipped U1V4 U2V4 U1V8 --rounds 7 --launches 10 --out $O/ab_bf16_shard4.json >> $O/ab.txt 2>&1
rc=$?
grep "^bf16" $O/ab.txt
exit $rc
