#!/bin/bash
# Round 5 profile set: rocprofv3 kernel stats of the default bench line, the
# config-4 FedAvg / median lines and the Krum line, beside their JSON lines.
set -o pipefail
O=gpurun_out/r05/d
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_cfg3.json 2> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg3 -o run \
      -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_cfg3.log 2>&1 \
 && timeout -k 10 300 python bench.py --config cfg4 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_cfg4.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --config cfg4 --op median --steps 5 --warmup 2 > $O/median_cfg4.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --op krum --steps 10 --warmup 3 > $O/krum_cfg3.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --config cfg5 --fedopt adam --steps 20 --warmup 5 > $O/cfg5_adam.json 2>> $O/bench.err
rc=$?
find $O -name '*kernel_trace.csv' -delete
for f in $O/bench_cfg3.json $O/bench_cfg4.json $O/median_cfg4.json $O/krum_cfg3.json $O/cfg5_adam.json; do python3 -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('$f'.split('/')[-1], round(d['ms_per_step'],4), r['kernel_ms_per_step'], r['achieved'], r['frac'])" 2>/dev/null; done
find $O -name '*kernel_stats.csv' | head -3
exit $rc
