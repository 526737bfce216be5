#!/bin/bash
# Re-check of the whole tree on a fresh box: GPU tests, smoke, headline bench,
# then a 2-rank rehearsal of bench.py's multi-process path (gloo, both ranks on
# the one GPU: RCCL refuses two ranks per device) for both partitionings.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r01e}
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
 && timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && timeout -k 10 300 $RUN bench.py --gpus 2 --backend gloo --config cfg5 --steps 5 --warmup 2 > gpurun_out/bench2_client_${TAG}.json 2> gpurun_out/bench2_client_${TAG}.err \
 && timeout -k 10 300 $RUN bench.py --gpus 2 --backend gloo --config cfg5 --mode param --steps 5 --warmup 2 > gpurun_out/bench2_param_${TAG}.json 2> gpurun_out/bench2_param_${TAG}.err \
 && timeout -k 10 300 $RUN bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > gpurun_out/bench2_cfg3_${TAG}.json 2> gpurun_out/bench2_cfg3_${TAG}.err
rc=$?
tail -2 gpurun_out/pytest_${TAG}.log; cat gpurun_out/smoke_${TAG}.log
for f in bench bench2_client bench2_param bench2_cfg3; do cat gpurun_out/${f}_${TAG}.json 2>/dev/null | cut -c1-400; done
exit $rc
