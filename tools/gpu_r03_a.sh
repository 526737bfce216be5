#!/bin/bash
# Round 3, first GPU pass: the whole -m gpu suite, the 1-GPU bench, and a
# 2-rank gloo rehearsal of the strong-scaling bench modes on the one GPU.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03/gputest.log 2>&1 || { tail -30 gpurun_out/r03/gputest.log; exit 1; }
tail -3 gpurun_out/r03/gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03/bench1.json 2> gpurun_out/r03/bench1.err || exit 1
cat gpurun_out/r03/bench1.json
for args in "--mode param" "--mode client" "--mode param --config cfg5 --fedopt sgd" "--mode client --config cfg5 --fedopt sgd"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo $args \
      > gpurun_out/r03/gloo2_$tag.json 2> gpurun_out/r03/gloo2_$tag.err || { tail -20 gpurun_out/r03/gloo2_$tag.err; exit 1; }
  cat gpurun_out/r03/gloo2_$tag.json
done
