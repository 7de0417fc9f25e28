#!/bin/bash
set -o pipefail
# Round 6, pass aj: the whole -m gpu suite once more on the final tree (stability of the 8-rank
# shapes; a device-wait timeout would now print the waiting launch and the slot re-read from memory)
O=gpurun_out/r06aj
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
grep -n "FAILED\|the waited slot now\|last launches with flag epochs" $O/pytest.log | head -20
exit $rc
