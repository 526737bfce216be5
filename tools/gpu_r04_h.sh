#!/bin/bash
# Round 4: the multi-device ingest through one native gather per client
# (fedagg_host_gather): GPU suite, then the interleaved ingest / host-round
# timings at G = 1, 2, 4 shards on the box's GPU.
set -o pipefail
O=gpurun_out/r04/h
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 600 python tools/multidev_bench.py --clients 32 --reps 4 --ingest --out $O/multidev_bench.json > $O/multidev_bench.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep "ingest\|host \|device " $O/multidev_bench.log
exit $rc
