set -o pipefail
# Round 5, pass aa: reduce-scatter operands up to 4 KiB element by element (MV2AMD_RS_SCALAR_MAX
# default 4096): the collective and MPICH coll tests
O=gpurun_out/r05aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread \
  tests/test_gpu_collectives_mp.py tests/test_gpu_mpich_coll_suite.py tests/test_gpu_multinode_mp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
