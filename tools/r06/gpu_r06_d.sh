#!/bin/bash
# Round 6, session d: host issue time of one-process rounds over G shards (FedOpt config 5, FedAvg config 3).
set -o pipefail
OUT=gpurun_out/r06/d
mkdir -p $OUT
timeout -k 10 300 python tools/probe_fedopt_issue.py $OUT/fedopt_issue.json > $OUT/fedopt_issue.txt 2>&1 \
 && timeout -k 10 300 python -m tools.probe_inprocess_issue > $OUT/inprocess_issue.txt 2>&1
rc=$?
cat $OUT/fedopt_issue.txt | head -60; cat $OUT/inprocess_issue.txt | head -8
exit $rc
