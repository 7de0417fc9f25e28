set -o pipefail
# Round 4, pass i: the one-node collectives after the nonblocking / block non-commutative
# reduce-scatter restatement (user-op cases via inb / block / iblock)
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 280 --timeout-method thread tests/test_gpu_collectives_mp.py -k "test_collectives_multiprocess or test_mv2_selection_knobs" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
