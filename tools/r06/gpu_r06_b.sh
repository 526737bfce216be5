#!/bin/bash
# Round 6, session b: the six OptRepo optimizers fused (tests + config-5 bench lines), FedOpt / SP aliasing,
# the one-call device round (config 1 on device dicts), set_model_params' load overrides.
set -o pipefail
OUT=gpurun_out/r06/b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fedopt_optrepo.py \
      tests/test_gpu_device_round.py tests/test_gpu_fedopt.py tests/test_simulation.py tests/test_gpu_multidev_fedopt.py \
      tests/test_gpu_host_copy.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/small_agg_bench.py $OUT/small_agg.json > $OUT/small_agg.txt 2>&1 || exit $?
cat $OUT/small_agg.txt
for o in adamax nadam radam adadelta asgd rprop adam sgd; do
  timeout -k 10 120 python bench.py --config cfg5 --fedopt $o --steps 30 --no-cpu-baseline > $OUT/cfg5_$o.json 2> $OUT/cfg5_$o.err || exit $?
done
python - <<'PY'
import json
for o in "adamax nadam radam adadelta asgd rprop adam sgd".split():
    d = json.load(open(f"gpurun_out/r06/b/cfg5_{o}.json"))
    r = d["roofline"]
    print(o, round(d["ms_per_step"], 4), r["kernel_ms_per_step"], r["achieved"], r["frac"])
PY
