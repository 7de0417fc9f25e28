#!/bin/bash
set -o pipefail
# Round 6, pass y: k_reduce_local_tiny without the wait for its stores before the release (and its arguments fetched in one batch)
O=gpurun_out/r06y
mkdir -p $O
timeout -k 10 90 tools/diag/rl_lat aql 5000 > $O/aql_variants.jsonl 2>&1 || { cat $O/aql_variants.jsonl; exit 1; }
grep -v "agent/none" $O/aql_variants.jsonl
for k in 1 2 3; do timeout -k 10 60 tools/diag/rl_lat lib 5000 | tee -a $O/lib.jsonl; done
