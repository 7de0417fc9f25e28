set -o pipefail
# Round 4, pass a: the whole -m gpu suite (12x4 point-to-point back in the default list, full-size
# configs at n = 4, 1 GiB allreduce at n = 4 / 8), once.
O=gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
