set -o pipefail
# Round 3, pass aa: nonblocking Iallreduce / Ireduce schedules above 8 ranks
# schedules, leaders' recursive doubling over 12 nodes), then the rest of the multi-node file.
O=gpurun_out/r03aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_multinode_mp.py -k "more_than_eight" > $O/pytest_9.log 2>&1 || { echo "tests failed"; tail -80 $O/pytest_9.log; exit 1; }
tail -3 $O/pytest_9.log
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_multinode_mp.py -k "not more_than_eight" > $O/pytest_mn.log 2>&1 || { echo "tests failed"; tail -80 $O/pytest_mn.log; exit 1; }
tail -3 $O/pytest_mn.log
