#!/bin/bash
# Round 5: fp32-accumulated bf16 at U1V4 / U1V8.  Large-size tests, the whole
# GPU suite, and the shipped dispatch against both shapes.
set -o pipefail
O=gpurun_out/r05/u
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_large.log 2>&1 || ok=1
[ $ok = 0 ] && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || ok=1; }
if [ $ok = 0 ]; then
for KN in "512 86567656" "512 43283828" "512 21641914" "64 86567656"; do
  set -- $KN
  timeout -k 10 200 python -u tools/ab_backtoback.py --dtype bf16acc32 --K $1 --N $2 --variants shipped U1V8 U1V4 --rounds 5 --launches 10 >> $O/ab.txt 2>&1 || { ok=1; break; }
done
fi
[ $ok = 0 ] && { timeout -k 10 300 python bench.py --config cfg4 --acc fp32 --no-cpu-baseline > $O/bench_cfg4_acc32.json 2> $O/bench.err || ok=1; }
grep -cE "PASSED" $O/pytest_large.log; grep -E "FAILED|Error" $O/pytest_large.log | head -5
tail -1 $O/pytest_gpu.log
grep "^bf16" $O/ab.txt
cut -c1-200 $O/bench_cfg4_acc32.json
exit $ok
