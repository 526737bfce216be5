#!/bin/bash
# Gram A/B over chunk-table piece lengths: bash tools/gpu_gram_chunks.sh OUTDIR CHUNK... -- TAG=-DFLAG=V ...
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
chunks=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do chunks+=("$1"); shift; done
shift
args=()
for v in "$@"; do args+=(--variant "$v"); done
rc=0
for ch in "${chunks[@]}"; do
  GRAM_AB_DIR=tools/_abbuild timeout -k 10 300 python tools/gram_variants.py --rounds 7 --chunk $ch \
      --out $O/gram_chunk$ch.json "${args[@]}" > $O/gram_chunk$ch.log 2>&1 || { rc=$?; break; }
  echo "chunk $ch"; grep -v amdgpu.ids $O/gram_chunk$ch.log | tail -6
done
exit $rc
