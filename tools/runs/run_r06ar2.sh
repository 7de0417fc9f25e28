#!/bin/bash
set -o pipefail
# Round 6, pass ar2: flag polls as never-writing atomics -- the whole -m gpu suite three more times
# (stall at the 8-rank soak: 3 of 10 suites before the change)
O=gpurun_out/r06ar2
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2 3; do
  timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest$k.log 2>&1; rc=$?
  tail -1 $O/pytest$k.log
  grep -n "FAILED\|the waited slot now\|waited for epoch" $O/pytest$k.log | cut -c1-300 | head -20
  [ $rc -eq 0 ] || exit $rc
done
