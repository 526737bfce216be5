#!/bin/bash
# Round 3: full GPU suite, many-client probes (16-bit tiny tile change),
# multi-device splitting overhead, headline bench + rocprofv3 stats.
set -o pipefail
O=gpurun_out/r03/final1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { echo "== $*" >&2; "$@"; }
run timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -2 $O/test.log
run timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
for d in bf16 f16 f32; do
  run timeout -k 10 200 python tools/manyclient_probe.py --dtype $d --out r03/final1/manyclient_$d > $O/manyclient_$d.log 2>&1 \
    || { tail $O/manyclient_$d.log; exit 1; }
done
run timeout -k 10 300 python tools/multidev_bench.py --clients 32 --reps 3 > $O/multidev.log 2>&1 || { tail $O/multidev.log; exit 1; }
cp gpurun_out/r03/multidev_bench.json $O/
run timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench \
      -- python3 bench.py --no-cpu-baseline > $O/prof_bench.log 2>&1 || { tail $O/prof_bench.log; exit 1; }
echo done
