#!/bin/bash
set -o pipefail
# Round 6, pass j: the library's HSA-queue fast path profiled (entry -> doorbell, doorbell -> word)
# with the packet's acquire at system (default) and agent scope, beside the HIP launch and the raw
# AQL floor with a system acquire and no release
O=gpurun_out/r06j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 tools/diag/rl_lat aql 5000 | tee $O/aql_floor.jsonl || exit 1
MV2AMD_HOST_PROFILE=200 timeout -k 10 60 tools/diag/rl_lat lib 5000 2>&1 | tee $O/lib_aql.txt || exit 1
MV2AMD_HOST_PROFILE=200 MV2AMD_AQL_ACQUIRE=1 timeout -k 10 60 tools/diag/rl_lat lib 5000 2>&1 | tee $O/lib_aql_agent.txt || exit 1
MV2AMD_HOST_PROFILE=200 MV2AMD_AQL=0 timeout -k 10 60 tools/diag/rl_lat lib 5000 2>&1 | tee $O/lib_hip.txt || exit 1
