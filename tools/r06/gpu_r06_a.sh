#!/bin/bash
# Round 6, session a: the restructured bench.py on the one-GPU box.
#   1. the default line (N = 1) is unchanged
#   2. --gpus 4 and --gpus 8 on gloo: every nested leg (cfg3 exchange / inprocess, cfg4 param / exchange /
#      inprocess, cfg5 sharded / one-process FedOpt) as a rehearsal, within the job budget
#   3. the multi-rank GPU tests
set -o pipefail
OUT=gpurun_out/r06/a
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 > $OUT/bench1.json 2> $OUT/bench1.err \
 && timeout -k 10 420 python bench.py --gpus 4 --backend gloo > $OUT/gloo4.json 2> $OUT/gloo4.err \
 && timeout -k 10 420 python bench.py --gpus 8 --backend gloo --steps 20 > $OUT/gloo8.json 2> $OUT/gloo8.err \
 && timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_multidev_fedopt.py \
      tests/test_gpu_multirank.py > $OUT/pytest.log 2>&1
rc=$?
cat $OUT/bench1.json; tail -2 $OUT/pytest.log
exit $rc
