set -o pipefail
# Round 5, pass h: the whole -m gpu suite with the point-to-point copy kernels
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
