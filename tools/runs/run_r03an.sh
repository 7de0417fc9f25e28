set -o pipefail
# Round 3, pass an: rehearse r03ab's sequence — the 12-rank collective tests, then point-to-point
# at 3x4 — three times, every failed rank's log kept
O=gpurun_out/r03an
mkdir -p $O
export TMPDIR=/tmp
export MV2AMD_TEST_P2P_EXTRA=12x4
for i in 1 2 3; do
  timeout -k 10 500 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_multinode_mp.py tests/test_gpu_p2p_mp.py -k "more_than_eight or 12-4" > $O/pytest_$i.log 2>&1 || { echo "run $i failed"; grep -v "^E  *$" $O/pytest_$i.log | grep -n "rank\|rror\|assert\|timed out" | tail -80; exit 1; }
  tail -1 $O/pytest_$i.log
done
