#!/bin/bash
# Round 5: U1V8 against U1V4 / U2V4 over row lengths (the whole-key shards of
# config 4 at 2 / 4 / 8 GPUs are 43.3M / 21.6M / 10.8M elements).
set -o pipefail
O=gpurun_out/r05/q
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ok=0
for KN in "512 10820957" "512 12582912" "512 21641914" "512 25165824" "512 33554432" "512 43283828" "512 60000000" "256 21641914" "256 43283828"; do
  set -- $KN
  timeout -k 10 200 python -u tools/ab_backtoback.py --dtype bf16 --K $1 --N $2 --variants U1V8 U1V4 U2V4 --rounds 5 --launches 10 >> $O/ab.txt 2>&1 || { ok=1; break; }
done
for KN in "128 43283828" "128 21641914" "256 86567656" "64 43283828"; do
  set -- $KN
  [ $ok = 0 ] || break
  timeout -k 10 200 python -u tools/ab_backtoback.py --dtype bf16f32 --K $1 --N $2 --variants U1V8 U1V4 shipped --rounds 5 --launches 10 >> $O/ab.txt 2>&1 || { ok=1; break; }
done
grep "^bf16" $O/ab.txt
exit $ok
