#!/bin/bash
set -o pipefail
# Round 6, pass am: the whole -m gpu suite three times with long device waits refreshing their
# cached lines every 200 us (device_util.h wait_mask; r06al: a poll served a stale slot for 30 s),
# the soaks' refresh counts recorded per rank
O=gpurun_out/r06am
mkdir -p $O
export TMPDIR=/tmp
export MV2AMD_TEST_RECORD=$PWD/$O/records.jsonl
for k in 1 2 3; do
  timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest$k.log 2>&1; rc=$?
  tail -1 $O/pytest$k.log
  grep -n "FAILED\\|the waited slot now\\|last launches with flag epochs\\|waited for epoch" $O/pytest$k.log | cut -c1-300 | head -20
  [ $rc -eq 0 ] || exit $rc
done
grep soak $O/records.jsonl
