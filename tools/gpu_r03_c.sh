#!/bin/bash
# Round 3: whole -m gpu suite after the tile-threshold change and the new
# fixtures, then the mid-size sweep again (shipped should now lead), the
# 1-GPU bench, and the cfg5 FedOpt strong-scaling rehearsal.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03/gputest_c.log 2>&1 || { tail -40 gpurun_out/r03/gputest_c.log; exit 1; }
tail -2 gpurun_out/r03/gputest_c.log
timeout -k 10 300 python tools/tune_mid.py --rounds 25 > gpurun_out/r03/tune_mid_c.txt 2>&1 || exit 1
cut -c1-75 gpurun_out/r03/tune_mid_c.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03/bench1_c.json 2>&1 || exit 1
cat gpurun_out/r03/bench1_c.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --config cfg5 --fedopt sgd \
    > gpurun_out/r03/gloo2_cfg5_c.json 2> gpurun_out/r03/gloo2_cfg5_c.err || { tail -20 gpurun_out/r03/gloo2_cfg5_c.err; exit 1; }
cat gpurun_out/r03/gloo2_cfg5_c.json
