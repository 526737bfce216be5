#!/bin/bash
# Round 6, session f: one-process multi-GPU rounds issued in one native call (FedOpt and FedAvg),
# the whole GPU suite on that library, issue-time probes, config-5 line, 8-rank gloo rehearsal,
# smoke, the default bench line and its rocprofv3 summary.
set -o pipefail
OUT=gpurun_out/r06/f
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python tools/probe_fedopt_issue.py $OUT/fedopt_issue.json > $OUT/fedopt_issue.txt 2>&1 \
 && timeout -k 10 300 python -m tools.probe_inprocess_issue > $OUT/inprocess_issue.txt 2>&1 \
 && timeout -k 10 120 python bench.py --config cfg5 --fedopt sgd --steps 30 --no-cpu-baseline > $OUT/cfg5_sgd.json 2> $OUT/cfg5_sgd.err \
 && timeout -k 10 420 python bench.py --gpus 8 --backend gloo --steps 20 > $OUT/gloo8.json 2> $OUT/gloo8.err \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err \
 && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench \
      -- python3 bench.py --steps 25 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.log
rc=$?
tail -2 $OUT/pytest_gpu.log; head -5 $OUT/fedopt_issue.txt; head -9 $OUT/inprocess_issue.txt; cat $OUT/smoke.log; cat $OUT/bench.json
exit $rc
