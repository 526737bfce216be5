#!/bin/bash
# Round 5: bf16 reference-chain tile shapes after the packed rounding, at
# config 4's own shape (512 x 86.6M) and around it.  Every variant is checked
# bit for bit against the shipped dispatch inside the tool.
set -o pipefail
O=gpurun_out/r05/j
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u tools/tune_tiny.py --dtypes bf16 --K 512 128 64 --N 86567656 --rounds 9 --out $O/ab_bf16_vit.json > $O/ab_bf16_vit.txt 2>&1 \
 && timeout -k 10 300 python -u tools/tune_tiny.py --dtypes bf16 --K 512 256 --N 16777216 8388608 --rounds 9 --out $O/ab_bf16_mid.json > $O/ab_bf16_mid.txt 2>&1
rc=$?
cat $O/ab_bf16_vit.txt $O/ab_bf16_mid.txt | grep bf16 | cut -c1-90
exit $rc
