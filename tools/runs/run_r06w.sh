#!/bin/bash
set -o pipefail
# Round 6, pass w: the AQL word kernel's variants at acquire agent / release none -- system-release
# word, write-through payload + relaxed word, kernel-argument preloading -- beside the library call
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 90 tools/diag/rl_lat aql 5000 > $O/aql_variants.jsonl 2>&1 || { cat $O/aql_variants.jsonl; exit 1; }
cat $O/aql_variants.jsonl
timeout -k 10 60 tools/diag/rl_lat lib 5000 | tee $O/lib.jsonl
