#!/bin/bash
set -o pipefail
# Round 6, pass k: the library's HSA-queue path with and without its per-call HIP stream queries
# (MV2AMD_AQL_STREAM_CHECKS=0 is a measurement knob), system and agent acquire
O=gpurun_out/r06k
mkdir -p $O
export TMPDIR=/tmp
for acq in 2 1; do for chk in 1 0; do
  echo "== acquire $acq stream_checks $chk"
  MV2AMD_HOST_PROFILE=200 MV2AMD_AQL_ACQUIRE=$acq MV2AMD_AQL_STREAM_CHECKS=$chk timeout -k 10 60 tools/diag/rl_lat lib 5000 2>&1 | tee -a $O/lib_variants.txt || exit 1
done; done
