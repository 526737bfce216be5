#!/bin/bash
# Round 5: bf16 reference chain in packed form (high-half rounding + step2).
# The whole GPU suite, the in-process A/B against the low-half form at
# config-4-sized rows, and the config 4 bench line with its rocprof stats.
set -o pipefail
O=gpurun_out/r05/i
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 400 python -u tools/tune_tiny.py --dtypes bf16 --K 128 32 --N 86567656 --rounds 9 --out $O/ab_bf16.json > $O/ab_bf16.txt 2>&1 \
 && timeout -k 10 400 python -u tools/tune_tiny.py --dtypes bf16 --K 512 --N 16777216 1000000 --rounds 9 --out $O/ab_bf16_k512.json > $O/ab_bf16_k512.txt 2>&1 \
 && timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 bench.py --config cfg4 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -delete
tail -2 $O/pytest_gpu.log
cat $O/ab_bf16.txt $O/ab_bf16_k512.txt 2>/dev/null | cut -c1-200
cat $O/bench_cfg4.json 2>/dev/null | cut -c1-400
exit $rc
