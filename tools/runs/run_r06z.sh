#!/bin/bash
set -o pipefail
# Round 6, pass z: host costs inside the 8-byte MPI_Reduce_local (pointer classification, API layer,
# the HSA-queue path's entry -> doorbell -> word split)
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 60 tools/diag/rl_lat lib 5000 | tee $O/lib.jsonl
MV2AMD_HOST_PROFILE=200 timeout -k 10 60 tools/diag/rl_lat lib 5000 2>&1 | tee $O/lib_hostprof.txt
