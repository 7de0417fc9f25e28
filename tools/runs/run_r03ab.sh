set -o pipefail
# Round 3, pass ab: the whole -m gpu suite after the message-schedule work (flat allreduce /
# reduce-scatter / nonblocking schedules above 8 ranks, basic reduce-scatter across nodes).
O=gpurun_out/r03ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -80 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
