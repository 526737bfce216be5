#!/bin/bash
# Non-temporal vs plain loads in the K <= 128 median kernels (config 3 / 4 shapes).
set -o pipefail
O=gpurun_out/r03/cols_nt
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MEDIAN_AB_SHAPES=cols MEDIAN_AB_REPS=12 MEDIAN_AB_VARIANTS="nt=-DFEDAGG_COLS_NT=1;plain=-DFEDAGG_COLS_NT=0" \
  timeout -k 10 600 python tools/median_ab.py $O/ab.json > $O/ab.log 2>&1; rc=$?
cat $O/ab.log; exit $rc
