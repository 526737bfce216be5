set -o pipefail
mkdir -p gpurun_out
for cfg in "4,12,48:96" "4,12,48:256" "4,12,48:32" "2,6,24:96" "8,24:96" "4,12:256" "4,12,48:96"; do
  ch=${cfg%%:*}; tl=${cfg##*:}
  timeout -k 10 120 python tools/devdict_bench.py --reps 30 --chunks $ch --tail $tl > gpurun_out/sw.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/devdict.json'));print('$cfg', round(d['wall_to_done_ms_median'],3), round(d['host_enqueue_ms_median'],3), round(d['gpu_window_ms_median'],3))" | tee -a gpurun_out/sweep.txt
done
