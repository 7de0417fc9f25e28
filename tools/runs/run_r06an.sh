#!/bin/bash
set -o pipefail
# Round 6, pass an: diagnosis of the r06u / r06al / r06am stall -- small allreduces at 8 ranks with
# 4 MiB of fresh pageable host memory uploaded and freed between calls, against one kept array
O=gpurun_out/r06an
mkdir -p $O
export TMPDIR=/tmp
for cfg in "8 2000 4194304 fresh all" "8 2000 4194304 kept all" "8 2000 33554432 fresh all" "2 3000 33554432 fresh all"; do
  echo "== $cfg $(date +%T)"
  timeout -k 10 420 python -u tools/diag/churn_probe.py $cfg >> $O/churn.jsonl 2> $O/churn_last.err || { echo "probe failed rc $?"; tail -20 $O/churn_last.err; exit 1; }
  tail -1 $O/churn.jsonl | cut -c1-700
done
