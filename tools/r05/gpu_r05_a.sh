#!/bin/bash
# Round 5, first check: the aliasing parity tests on the GPU, and bench.py's
# self-launch (`--gpus 2` without torchrun, gloo: two ranks on the box's one
# GPU) with the nested one-process measurement.
set -o pipefail
O=gpurun_out/r05/a
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 \
 && timeout -k 10 420 python bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 > $O/gloo2_cfg3.json 2> $O/gloo2.err
rc=$?
tail -1 $O/pytest_parity.log
cat $O/gloo2_cfg3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['ms_per_step'], json.dumps(d.get('inprocess'))[:600], json.dumps(d.get('exchange'))[:300])"
exit $rc
