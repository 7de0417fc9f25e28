#!/bin/bash
set -o pipefail
# Round 6, pass i: the raw AQL floor (tools/diag/rl_lat aql: a one-wave kernel dispatched by hand into
# an HSA queue, three fence-scope settings) and the host cost of hipStreamQuery, the checks the
# library's fast path makes; why the fast path measured slower than the HIP launch (r06h)
O=gpurun_out/r06i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 tools/diag/rl_lat aql 5000 | tee $O/aql_floor.jsonl || exit 1
timeout -k 10 60 tools/diag/rl_lat floor 5000 | tee $O/floor.jsonl
