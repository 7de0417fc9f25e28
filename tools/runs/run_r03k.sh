set -o pipefail
# Round 3, pass k: point-to-point across emulated nodes (rank mesh), the one-node p2p tests,
# the multi-node collectives again (mesh set up at MPI_Init, internal tag context).
O=gpurun_out/r03k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_p2p_mp.py > $O/pytest_p2p.log 2>&1 || { echo "p2p tests failed"; tail -150 $O/pytest_p2p.log; exit 1; }
tail -3 $O/pytest_p2p.log
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_multinode_mp.py > $O/pytest_mn.log 2>&1 || { echo "multinode tests failed"; tail -120 $O/pytest_mn.log; exit 1; }
tail -3 $O/pytest_mn.log
