#!/bin/bash
# Round 6, session i: the fp32 FedAvg tile variants (tuning build, device weights) against the
# shipped dispatch (device and kernel-argument weights) at the per-device sizes of configs 3 and 5
# split over 1-8 GPUs, where tools/shard_rates.py found the shipped tiles at 0.69-0.78 of HBM;
# then shard_rates again with config 4 fixed.
set -o pipefail
OUT=gpurun_out/r06/i
mkdir -p $OUT
for kn in "128 3201269" "128 6402538" "64 4194304" "64 1048576" "64 524288"; do
  set -- $kn
  timeout -k 10 240 python tools/tune_wsum.py --K $1 --N $2 --rounds 15 > $OUT/tune_K$1_N$2.txt 2>&1 || exit 1
done
timeout -k 10 300 python tools/shard_rates.py > $OUT/shard_rates.txt 2>&1
rc=$?
for f in $OUT/tune_*.txt; do echo "== $f"; grep -v bitwise $f; done; grep -c MISMATCH $OUT/tune_*.txt; cat $OUT/shard_rates.txt
exit $rc
