#!/bin/bash
# Round 4, last GPU check: the multi-rank bench path rehearsed with gloo on
# the box's one GPU (2 ranks; config 3 and config 4 at BASELINE's client
# counts, both partitionings in one line), the FedOpt config-5 line, and the
# multi-device FedOpt tests.
set -o pipefail
O=gpurun_out/r04/final3
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > $O/gloo2_cfg3.json 2> $O/gloo2_cfg3.err \
 && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29534 bench.py --gpus 2 --backend gloo --config cfg5 --fedopt adam --steps 3 --warmup 1 \
    > $O/gloo2_cfg5_adam.json 2> $O/gloo2_cfg5.err \
 && timeout -k 10 300 python bench.py --config cfg5 --fedopt adam --steps 20 --no-cpu-baseline > $O/bench_cfg5_adam.json 2> $O/bench.err \
 && timeout -k 10 300 python -u -m pytest tests/test_gpu_multidev_fedopt.py tests/test_gpu_fedopt.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest_fedopt.log 2>&1
rc=$?
for f in $O/gloo2_cfg3.json $O/gloo2_cfg5_adam.json $O/bench_cfg5_adam.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
e=d.get('exchange') or {}
print('$f'.split('/')[-1], d['n_gpus'], d['config'].get('clients_total'), round(d['ms_per_step'],3), d['roofline']['frac'], e.get('mode'), e.get('backend'), e.get('clients'), e.get('ms_per_step'))
" 2>&1 | tail -1; done
tail -1 $O/pytest_fedopt.log
exit $rc
