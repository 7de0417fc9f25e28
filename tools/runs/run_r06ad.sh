#!/bin/bash
set -o pipefail
# Round 6, pass ad: the 8-rank soak that timed out once (r06u), behind the two smaller soaks as in
# the suite, then once at 40,000 calls -- a timeout now prints the launch that waited and the
# waited slot as a copy re-reads it from memory
O=gpurun_out/r06ad
mkdir -p $O
T="tests/test_gpu_collectives_mp.py::test_soak_thousands_of_calls"
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread "$T[2-16000-11-env0-None]" "$T[4-10000-12-env1-None]" "$T[8-5000-13-env2-None]" > $O/soaks.log 2>&1 || { echo "soaks failed"; grep -n "error\|Error" $O/soaks.log | head -60; exit 1; }
tail -1 $O/soaks.log
MV2AMD_SOAK_CALLS=40000 timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 560 --timeout-method thread "$T[8-5000-13-env2-None]" > $O/soak8_40k.log 2>&1 || { echo "long soak failed"; grep -n "error\|Error" $O/soak8_40k.log | head -60; exit 1; }
tail -1 $O/soak8_40k.log
