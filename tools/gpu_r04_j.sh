#!/bin/bash
# Round 4: FedOpt over several GPUs of one process (MultiDeviceFedOptServer,
# all shards on the box's one GPU) against the one-device server.
set -o pipefail
O=gpurun_out/r04/j
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_multidev_fedopt.py tests/test_gpu_fedopt.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -25 $O/pytest.log
exit $rc
