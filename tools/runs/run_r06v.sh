#!/bin/bash
set -o pipefail
# Round 6, pass v: the 8-rank soak that timed out once in r06u (a peer's flag slot read an epoch
# older than one it had already passed), twice, with the timeout report's new lines (the launch
# that waited, the slot as it is in memory now)
O=gpurun_out/r06v
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 420 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread \
    "tests/test_gpu_collectives_mp.py::test_soak_thousands_of_calls[8-5000-13-env2-None]" > $O/soak$k.log 2>&1 || { echo "soak $k failed"; grep -n "error" $O/soak$k.log | head -80; exit 1; }
  tail -1 $O/soak$k.log
done
