set -o pipefail
# Round 4, pass h: the multi-node tests after MPI_Reduce's multi-node tables (emulated nodes on the one GPU)
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests/test_gpu_multinode_mp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
