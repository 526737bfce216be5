set -o pipefail
mkdir -p gpurun_out/r02p
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_defenses.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02p/tests.log 2>&1 \
 && B="python bench.py --no-cpu-baseline" \
 && timeout -k 10 300 $B --op krum --steps 5 --warmup 1 > gpurun_out/r02p/bench_krum_cfg3.json 2> gpurun_out/r02p/bench.err \
 && timeout -k 10 300 $B --op dist2 --steps 20 > gpurun_out/r02p/bench_dist2_cfg3.json 2>> gpurun_out/r02p/bench.err \
 && timeout -k 10 300 $B --op clip --steps 20 > gpurun_out/r02p/bench_clip_cfg3.json 2>> gpurun_out/r02p/bench.err \
 && timeout -k 10 300 $B --op krum --config cfg5 --steps 20 > gpurun_out/r02p/bench_krum_cfg5.json 2>> gpurun_out/r02p/bench.err
rc=$?
tail -3 gpurun_out/r02p/tests.log
for f in gpurun_out/r02p/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['roofline'])"; done
exit $rc
