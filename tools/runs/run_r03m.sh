set -o pipefail
# Round 3, pass m: stream-ordered calls across nodes; one-node stream-ordered / graph regression.
O=gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_multinode_mp.py > $O/pytest_mn.log 2>&1 || { echo "multinode tests failed"; tail -120 $O/pytest_mn.log; exit 1; }
tail -3 $O/pytest_mn.log
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_collectives_mp.py -k "stream_ordered or graph" > $O/pytest_sq.log 2>&1 || { echo "stream tests failed"; tail -80 $O/pytest_sq.log; exit 1; }
tail -3 $O/pytest_sq.log
