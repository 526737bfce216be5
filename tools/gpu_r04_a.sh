#!/bin/bash
# Round 4, first GPU session: the GPU suite, the headline bench, config 4 at
# BASELINE's 512 clients (FedAvg, both accumulation modes) with rocprofv3
# kernel stats and the two PMC traffic passes, and a gloo rehearsal of the
# two-rank line (parameter axis + the nested client-axis exchange).
# Each GPU step runs under its own time limit; the chain stops at the first failure.
set -o pipefail
O=gpurun_out/r04/a
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
pmc() {  # key, kernel filter, bench args...
  local name=$1 kern=$2; shift 2
  local tag=${name//[:@]/_}
  local alg
  alg=$(python3 -c "import json; print(json.load(open('$O/bench_${tag}.json'))['roofline']['alg_bytes_per_step'])") || return 1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_${tag} -o b \
    -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/fetch_${tag}.log 2>&1 || return 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_${tag} -o b \
    -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/write_${tag}.log 2>&1 || return 1
  python3 tools/pmc_traffic.py --fetch $O/fetch_${tag}/b_counter_collection.csv \
    --write $O/write_${tag}/b_counter_collection.csv --key "${name}" --kernel "${kern}" \
    --alg-bytes "${alg}" --out $O/pmc_traffic.json
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && hipcc --offload-arch=gfx950 -O3 -o $O/valu_rate_probe tools/valu_rate_probe.hip > /dev/null 2>&1 \
 && VALU_PROBE_SAD=1 timeout -k 10 120 $O/valu_rate_probe > $O/valu_rate_probe_sad.txt 2>&1 \
 && timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench.err \
 && timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline > $O/bench_cfg4_single_K512.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --config cfg4 --acc fp32 --no-cpu-baseline > $O/bench_cfg4_single_acc32_K512.json 2>> $O/bench.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg4 -o bench \
      -- python3 bench.py --config cfg4 --steps 20 --no-cpu-baseline > $O/prof_cfg4.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg4_acc32 -o bench \
      -- python3 bench.py --config cfg4 --acc fp32 --steps 20 --no-cpu-baseline > $O/prof_cfg4_acc32.log 2>&1 \
 && pmc cfg4:single@K512 OpBF16Ref --config cfg4 \
 && pmc cfg4:single:acc32@K512 OpBF16Acc32 --config cfg4 --acc fp32 \
 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29531 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > $O/gloo2_cfg3.json 2> $O/gloo2_cfg3.err
rc=$?
find $O -name '*kernel_trace.csv' -delete
rm -f $O/valu_rate_probe
cat $O/valu_rate_probe_sad.txt 2>/dev/null
tail -3 $O/pytest_gpu.log
for f in $O/bench_*.json $O/gloo2_cfg3.json; do echo "== $f"; python3 -c "
import json,sys
for l in open('$f'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']
        print(d['ms_per_step'], r['kernel_ms_per_step'], r['achieved'], r['frac'], r['traffic'], d['config']['clients_total'], (d.get('cpu_baseline') or {}).get('ms_per_aggregation'), json.dumps(d.get('exchange')))
" 2>/dev/null; done
cat $O/pmc_traffic.json 2>/dev/null
exit $rc
