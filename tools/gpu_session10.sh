#!/bin/bash
# Sharded FedOpt (config 5 over several GPUs): GPU tests, then a 2-rank gloo
# rehearsal of bench.py --fedopt on the one GPU.
set -o pipefail
mkdir -p gpurun_out
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fedopt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_shfo.log 2>&1 \
 && timeout -k 10 300 $RUN bench.py --gpus 2 --backend gloo --config cfg5 --fedopt sgd --steps 5 --warmup 2 > gpurun_out/bench2_fedopt.json 2> gpurun_out/bench2_fedopt.err \
 && timeout -k 10 300 $RUN bench.py --gpus 2 --backend gloo --config cfg5 --fedopt adam --steps 5 --warmup 2 > gpurun_out/bench2_fedopt_adam.json 2>> gpurun_out/bench2_fedopt.err
rc=$?
tail -3 gpurun_out/pytest_shfo.log; grep -E "^E " gpurun_out/pytest_shfo.log | head -5; tail -3 gpurun_out/bench2_fedopt.err
cut -c1-300 gpurun_out/bench2_fedopt.json gpurun_out/bench2_fedopt_adam.json
exit $rc
