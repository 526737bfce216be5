#!/bin/bash
# Round 6, session e: FedOpt rounds issued through one batched native call (fedagg_wsum_fedopt_batch):
# the FedOpt GPU tests, the issue-time probes, config-5 lines and the 8-shard rehearsal of the nested legs.
set -o pipefail
OUT=gpurun_out/r06/e
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fedopt.py \
      tests/test_gpu_fedopt_optrepo.py tests/test_gpu_multidev_fedopt.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py \
      tests/test_gpu_multirank.py tests/test_c_abi.py > $OUT/pytest.log 2>&1 \
 && timeout -k 10 300 python tools/probe_fedopt_issue.py $OUT/fedopt_issue.json > $OUT/fedopt_issue.txt 2>&1 \
 && timeout -k 10 300 python -m tools.probe_inprocess_issue > $OUT/inprocess_issue.txt 2>&1 \
 && timeout -k 10 120 python bench.py --config cfg5 --fedopt sgd --steps 30 --no-cpu-baseline > $OUT/cfg5_sgd.json 2> $OUT/cfg5_sgd.err \
 && timeout -k 10 420 python bench.py --gpus 8 --backend gloo --steps 20 > $OUT/gloo8.json 2> $OUT/gloo8.err
rc=$?
tail -2 $OUT/pytest.log; head -5 $OUT/fedopt_issue.txt; head -5 $OUT/inprocess_issue.txt
exit $rc
