#!/bin/bash
# Round 5: U1V8 dispatched by last-round fill.  Whole GPU suite, then the
# shipped dispatch against both shapes at the lengths of r05/q, and the
# config 4 bench line.
set -o pipefail
O=gpurun_out/r05/s
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || ok=1
tail -1 $O/pytest_gpu.log
if [ $ok = 0 ]; then
for KN in "bf16 512 86567656" "bf16 512 43283828" "bf16 512 21641914" "bf16 512 33554432" "bf16f32 128 86567656" "bf16f32 128 43283828" "bf16f32 128 21641914" "bf16f32 128 10820957"; do
  set -- $KN
  timeout -k 10 200 python -u tools/ab_backtoback.py --dtype $1 --K $2 --N $3 --variants shipped U1V8 U1V4 --rounds 5 --launches 10 >> $O/ab.txt 2>&1 || { ok=1; break; }
done
fi
[ $ok = 0 ] && { timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench.err || ok=1; }
grep "^bf16" $O/ab.txt
cut -c1-300 $O/bench_cfg4.json
exit $ok
