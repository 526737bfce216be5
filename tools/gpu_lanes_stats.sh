#!/bin/bash
# rocprofv3 kernel stats for the median at 512 clients (config 4 bf16,
# config 3 rows fp32), next to the bench lines of the same commands.
set -o pipefail
O=gpurun_out/r03/lanes_stats
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in cfg4 cfg3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -o b \
    -- python3 bench.py --op median --config $cfg --clients 512 --steps 10 --warmup 2 --no-cpu-baseline \
    > $O/bench_${cfg}_k512.json 2> $O/prof_$cfg.err || exit 1
  cat $O/bench_${cfg}_k512.json
done
find $O -name '*kernel_trace.csv' -delete
for cfg in cfg4 cfg3; do grep -h median $O/prof_$cfg/b_kernel_stats.csv | cut -c1-200; done
