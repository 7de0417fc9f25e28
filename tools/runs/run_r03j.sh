set -o pipefail
# Round 3, pass j: multi-node restatements (table intra/inter functions, flat reduce-scatter over
# the job, user ops across nodes) and the one-node user-op tests around them.
O=gpurun_out/r03j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_multinode_mp.py > $O/pytest_mn.log 2>&1 || { echo "multinode tests failed"; tail -120 $O/pytest_mn.log; exit 1; }
tail -3 $O/pytest_mn.log
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_collectives_mp.py -k "user or x87 or reduce_scatter" > $O/pytest_user.log 2>&1 || { echo "user tests failed"; tail -80 $O/pytest_user.log; exit 1; }
tail -3 $O/pytest_user.log
