#!/bin/bash
set -o pipefail
# Round 6, pass ao: flag polls as never-writing atomics (performed at memory) -- OSU 8 B .. 2 KiB at
# 2 shared ranks A/B (A = the plain-load poll in abtest/), then the whole -m gpu suite twice
O=gpurun_out/r06ao
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export LD_LIBRARY_PATH=$PWD/abtest; else unset LD_LIBRARY_PATH; fi
    timeout -k 10 150 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 140 tools/osu/osu_coll -c all -m 8:2048 -f 16 -i 2000 -x 200 -v > $O/osu_${v}$k.txt 2>&1 || { tail -20 $O/osu_${v}$k.txt; exit 1; }
    echo "== $v$k $(grep -v '^JSON\|^#\|^\[' $O/osu_${v}$k.txt | awk '{printf "%s:%s ", $1, $2}' | cut -c1-300)"
  done
done
unset LD_LIBRARY_PATH
for k in 1 2; do
  timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest$k.log 2>&1; rc=$?
  tail -1 $O/pytest$k.log
  grep -n "FAILED\|the waited slot now\|waited for epoch" $O/pytest$k.log | cut -c1-300 | head -20
  [ $rc -eq 0 ] || exit $rc
done
