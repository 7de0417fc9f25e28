set -o pipefail
# Round 3, pass aj: host-op reduce-scatter above 8 ranks (basic / halving / ring for this rank's block)
O=gpurun_out/r03aj
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_multinode_mp.py -k "user_ops" > $O/pytest.log 2>&1 || { echo "tests failed"; grep -v "^E  *$" $O/pytest.log | tail -80; exit 1; }
tail -12 $O/pytest.log
