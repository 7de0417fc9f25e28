#!/bin/bash
set -o pipefail
# Round 6, pass al: the whole -m gpu suite twice more on the final tree (stability of the 8-rank
# shapes across suites)
O=gpurun_out/r06al
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest$k.log 2>&1; rc=$?
  tail -1 $O/pytest$k.log
  grep -n "FAILED\|the waited slot now\|last launches with flag epochs" $O/pytest$k.log | head -20
  [ $rc -eq 0 ] || exit $rc
done
