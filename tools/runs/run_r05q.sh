set -o pipefail
# Round 5, pass q: the reference's argument checks (buffer aliasing / MPI_IN_PLACE / null buffers,
# uncommitted types, MPI_Pack's space check) and the suites they could disturb
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_collectives_mp.py -k "argument_checks or derived or enqueue or graph or vector or nonblocking" \
  tests/test_gpu_reduce_local.py tests/test_gpu_pack.py tests/test_gpu_mpich_datatype_suite.py tests/test_gpu_mpich_coll_suite.py tests/test_gpu_p2p_mp.py \
  > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
