#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/tune_wsum.py --rounds 8 > gpurun_out/tune2.log 2>&1 \
 && timeout -k 10 300 python tools/hbm_probe.py > gpurun_out/hbm_probe.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o bench \
      -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o bench \
      -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 \
 && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_s2.json 2>gpurun_out/bench_s2.err
rc=$?
cat gpurun_out/tune2.log gpurun_out/hbm_probe.log gpurun_out/bench_s2.json 2>/dev/null | grep -v amdgpu.ids
echo "chain rc=$rc"
# RCCL with two ranks on one GPU: may be refused by RCCL; runs last, its own limit
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
   --master-port 29517 tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1
echo "rccl rc=$?"; grep -E "rank|Error|error|WARN" gpurun_out/rccl_probe.log | head -8
exit $rc
