#!/bin/bash
# Gram-kernel A/B on the GPU box: bash tools/gpu_gram_ab.sh OUTDIR TAG=-DFLAG=V ...
# (variants prebuilt here with tools/gram_variants.py --build into tools/_abbuild)
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
args=()
for v in "$@"; do args+=(--variant "$v"); done
GRAM_AB_DIR=tools/_abbuild timeout -k 10 300 python tools/gram_variants.py --rounds 9 --out $O/gram_variants.json \
    "${args[@]}" > $O/gram_variants.log 2>&1
rc=$?
grep -v amdgpu.ids $O/gram_variants.log | tail -12
exit $rc
