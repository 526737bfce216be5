#!/bin/bash
# Round 4: counting-median variants (values per lane R, accumulator chains) in one process.
set -o pipefail
O=gpurun_out/r04/c
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MEDIAN_AB_DIR=tools/_abbuild MEDIAN_AB_SHAPES=k512 \
  MEDIAN_AB_VARIANTS="r128c4=-DFEDAGG_SAD_CHAINS=4;hlc2=-DFEDAGG_PK16_COUNT_HL=1,-DFEDAGG_SAD_CHAINS=2;hlc4=-DFEDAGG_PK16_COUNT_HL=1,-DFEDAGG_SAD_CHAINS=4;net=-DFEDAGG_PK16_COUNT=0" \
  timeout -k 10 500 python tools/median_ab.py $O/median_ab_hl.json > $O/median_ab.log 2>&1
rc=$?
grep '^{' $O/median_ab.log
tail -3 $O/median_ab.log
exit $rc
