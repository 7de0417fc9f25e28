set -o pipefail
# Round 3, pass ad: the 12-rank (3x4) point-to-point + nonblocking test five times in one process
# (r03ab saw rank 0 fail with a leader's link closed; the test now prints every failed rank's log)
O=gpurun_out/r03ad
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_p2p_mp.py -k "12-4 or 10-1" > $O/pytest_$i.log 2>&1 || { echo "run $i failed"; grep -v "^E  *$" $O/pytest_$i.log | grep -n "rank\|Error\|error\|assert" | tail -80; exit 1; }
  tail -1 $O/pytest_$i.log
done
