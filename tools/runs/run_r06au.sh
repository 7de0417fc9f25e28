#!/bin/bash
set -o pipefail
# Round 6, pass au: the 8-byte Reduce_local beside the dispatch floor on the same box (box-to-box
# spread of the bench line's figure: 5.21-5.82 us across r06aa-r06at)
O=gpurun_out/r06au
mkdir -p $O
timeout -k 10 90 tools/diag/rl_lat aql 5000 > $O/aql.jsonl 2>&1 || { cat $O/aql.jsonl; exit 1; }
grep "agent/none: k_word system\|tiny (agent" $O/aql.jsonl
for k in 1 2; do timeout -k 10 60 tools/diag/rl_lat lib 5000 | grep "C loop" | tee -a $O/lib.jsonl; done
