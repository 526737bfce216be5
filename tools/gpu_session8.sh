set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_defense.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lanes.log 2>&1 \
 && timeout -k 10 300 python tools/median_probe.py --big-only > gpurun_out/median_probe_big.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_lanes.log; tail -40 gpurun_out/median_probe_big.log | head -12
exit $rc
