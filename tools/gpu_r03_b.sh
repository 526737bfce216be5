#!/bin/bash
# Round 3: tile configs at the per-rank sizes of strong scaling (config 3 at
# 2/4/8 ranks, config 5 at 2/4/8), and the fixed gloo rehearsal of cfg5 FedOpt.
set -o pipefail
mkdir -p gpurun_out/r03/tune
export TMPDIR=/tmp
for kn in "128 3201344" "128 6402624" "128 12805184" "64 524288" "64 1048576" "64 2097152"; do
  set -- $kn
  timeout -k 10 180 python tools/tune_wsum.py --K $1 --N $2 --rounds 8 > gpurun_out/r03/tune/K$1_N$2.txt 2>&1 \
      || { tail -5 gpurun_out/r03/tune/K$1_N$2.txt; exit 1; }
  grep -E "shipped|U4V4nt |U1V4nt |U16V1|U8V1nt_b64|U8V2nt_b64|U4V4nt_b64|b128|MISMATCH|read_probe" gpurun_out/r03/tune/K$1_N$2.txt
done
for args in "--mode param --config cfg5 --fedopt sgd" "--mode client --config cfg5 --fedopt sgd"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo $args \
      > gpurun_out/r03/gloo2_$tag.json 2> gpurun_out/r03/gloo2_$tag.err || { tail -20 gpurun_out/r03/gloo2_$tag.err; exit 1; }
  cat gpurun_out/r03/gloo2_$tag.json
done
