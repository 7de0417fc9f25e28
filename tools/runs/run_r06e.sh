#!/bin/bash
set -o pipefail
# Round 6, pass e: the 8-byte MPI_Reduce_local broken down: the platform floor
# without the library (empty kernel + stream sync; kernel raising a pinned host word with and
# without the system-scope release), the library call from C, with HIP_FORCE_DEV_KERNARG=1, with
# the host profile (entry -> launch, launch, launch -> word), and under rocprofv3 --kernel-trace;
# the library with and without the one-wave kernel for small operands (MV2AMD_RL_TINY_MAX=0)
O=gpurun_out/r06e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 tools/diag/rl_lat floor 5000 | tee $O/floor.jsonl && \
timeout -k 10 60 tools/diag/rl_lat lib 5000 | tee $O/lib.jsonl && \
MV2AMD_RL_TINY_MAX=0 timeout -k 10 60 tools/diag/rl_lat lib 5000 | tee $O/lib_notiny.jsonl && \
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 60 tools/diag/rl_lat floor 5000 | tee $O/floor_devkernarg.jsonl && \
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 60 tools/diag/rl_lat lib 5000 | tee $O/lib_devkernarg.jsonl && \
MV2AMD_HOST_PROFILE=200 timeout -k 10 60 tools/diag/rl_lat lib 5000 2>&1 | tee $O/lib_hostprof.txt && \
MV2AMD_SYNC=1 timeout -k 10 60 tools/diag/rl_lat lib 5000 | tee $O/lib_sync.jsonl && \
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o rl -- tools/diag/rl_lat lib 3000 > $O/trace.log 2>&1; echo "trace rc $?"
find $O/trace -name "*kernel_trace.csv" | head -2
