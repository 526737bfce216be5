#!/bin/bash
# Round 3: the centred-Gram Krum kernel (parity + speed), the dist2 reference
# row fix (A/B builds + PMC), rocprofv3 of the shipped krum / dist2.
set -o pipefail
O=gpurun_out/r03/gram3
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { echo "== $*" >&2; "$@"; }
B="python bench.py --no-cpu-baseline"
run timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_defenses.py -x -q --timeout 200 --timeout-method thread \
      > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -2 $O/test.log
run timeout -k 10 300 python tools/robust_variants.py --rounds 10 > $O/variants.txt 2>&1 || { tail $O/variants.txt; exit 1; }
cat $O/variants.txt | grep -E "clip|dist2|copy"
run timeout -k 10 300 $B --op krum --steps 10 --warmup 2 > $O/bench_krum_gram_cfg3.json 2> $O/bench.err \
 && run timeout -k 10 300 $B --op krum --pair-distance exact --steps 5 --warmup 1 > $O/bench_krum_exact_cfg3.json 2>> $O/bench.err \
 && run timeout -k 10 300 $B --op krum --config cfg5 --steps 20 > $O/bench_krum_gram_cfg5.json 2>> $O/bench.err \
 && run timeout -k 10 300 $B --op dist2 --steps 20 > $O/bench_dist2_cfg3.json 2>> $O/bench.err \
 && run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_krum -o krum \
      -- python3 bench.py --no-cpu-baseline --op krum --steps 10 --warmup 2 > $O/prof_krum.log 2>&1 \
 && run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dist2 -o dist2 \
      -- python3 bench.py --no-cpu-baseline --op dist2 --steps 20 > $O/prof_dist2.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch_dist2 -o dist2 \
      -- python3 bench.py --no-cpu-baseline --op dist2 --steps 3 --warmup 1 > $O/pmc_fetch_dist2.log 2>&1 \
 && run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write_dist2 -o dist2 \
      -- python3 bench.py --no-cpu-baseline --op dist2 --steps 3 --warmup 1 > $O/pmc_write_dist2.log 2>&1
rc=$?
for f in $O/bench_*.json; do echo $f; python3 -c "import json,sys;d=json.load(open('$f'));print(d['ms_per_step'],d['roofline'])"; done
exit $rc
