#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest9.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg2 -o cfg2 \
      -- python3 bench.py --config cfg2 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_cfg2.log 2>&1 \
 && timeout -k 10 300 python bench.py --config cfg4 --steps 20 --no-cpu-baseline > gpurun_out/bench_cfg4_ref.json 2>gpurun_out/b4.err \
 && timeout -k 10 300 python bench.py --config cfg4 --acc fp32 --steps 20 --no-cpu-baseline > gpurun_out/bench_cfg4_fp32.json 2>>gpurun_out/b4.err \
 && timeout -k 10 300 python bench.py --config cfg5 --fedopt --steps 100 --no-cpu-baseline > gpurun_out/bench_cfg5_fedopt.json 2>gpurun_out/b5.err \
 && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
      bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > gpurun_out/bench_gloo2.json 2>gpurun_out/bench_gloo2.err \
 && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 \
      bench.py --gpus 2 --backend gloo --mode param --steps 3 --warmup 1 > gpurun_out/bench_gloo2p.json 2>gpurun_out/bench_gloo2p.err
rc=$?
tail -2 gpurun_out/pytest9.log
grep -E "reduce_kernel" gpurun_out/prof_cfg2/cfg2_kernel_stats.csv | cut -c1-60,200-400
for f in bench_cfg4_ref bench_cfg4_fp32 bench_cfg5_fedopt bench_gloo2 bench_gloo2p; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['n_gpus'], 'ms/step %.4f'%d['ms_per_step'], 'kernel ms %.4f'%d['roofline']['kernel_ms_per_step'], 'GB/s', d['roofline']['achieved'], d['value'])" 2>&1 | tail -1; done
tail -3 gpurun_out/bench_gloo2.err
exit $rc
