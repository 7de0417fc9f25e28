set -o pipefail
# Round 3, pass ai: above 8 ranks incl. x87 long double (host-evaluated pt2pt_rs reduce-scatter,
# ring, IN_PLACE split) and user ops
O=gpurun_out/r03ai
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_multinode_mp.py -k "more_than_eight or user_ops" > $O/pytest.log 2>&1 || { echo "tests failed"; grep -v "^E  *$" $O/pytest.log | tail -80; exit 1; }
tail -12 $O/pytest.log
