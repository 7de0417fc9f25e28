set -o pipefail
# Round 3, pass l: the reference's MPICH collective tests on emulated nodes too.
O=gpurun_out/r03l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 320 --timeout-method thread tests/test_gpu_mpich_coll_suite.py > $O/pytest_suite.log 2>&1 || { echo "suite failed"; tail -150 $O/pytest_suite.log; exit 1; }
tail -3 $O/pytest_suite.log
