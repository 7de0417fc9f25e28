set -o pipefail
# Round 4, pass zf: the whole -m gpu suite on the final tree (host-window error path change)
O=gpurun_out/r04zf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
