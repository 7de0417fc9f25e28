set -o pipefail
# Round 4, pass p: the RD exchange with every allocation before the vote
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_collectives_mp.py tests/test_gpu_mpich_coll_suite.py -k "strided_vector or collectives_multiprocess or coll_suite" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -80 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
