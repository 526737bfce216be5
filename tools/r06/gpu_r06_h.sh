#!/bin/bash
# Round 6, session h: where config 5's per-client ingest loses to the link (tools/ingest_probe.py:
# H2D alone at 16.8 MB per copy, with / without the per-copy stream wait, pack + H2D in pieces,
# ring depth and pack threads), the plain FedAvg rate at the shard sizes of a split config 5, and
# the shipped kernels' rate at every per-device size of configs 3-5 split over 1-8 GPUs.
set -o pipefail
OUT=gpurun_out/r06/h
mkdir -p $OUT
timeout -k 10 300 python -m tools.ingest_probe --config cfg5 > $OUT/ingest_cfg5.txt 2>&1 \
 && timeout -k 10 300 python -m tools.ingest_probe --config cfg3 > $OUT/ingest_cfg3.txt 2>&1 \
 && timeout -k 10 300 python tools/ab_fused_shards.py tools/_abbuild/libfedagg_before_small_fused.so \
      fedml_amd/lib/libfedagg.so > $OUT/ab_fused_shards.txt 2>&1 \
 && timeout -k 10 300 python tools/shard_rates.py > $OUT/shard_rates.txt 2>&1
rc=$?
cat $OUT/ingest_cfg5.txt $OUT/ingest_cfg3.txt; grep avg $OUT/ab_fused_shards.txt; cat $OUT/shard_rates.txt
exit $rc
