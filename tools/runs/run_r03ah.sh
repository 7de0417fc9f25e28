set -o pipefail
# Round 3, pass ah: user ops across nodes above 8 ranks (12x1, 5x2): host-evaluated message
# schedules (recursive doubling, ring chunk, binomial, leaders' steps over 12 nodes)
O=gpurun_out/r03ah
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_multinode_mp.py -k "user_ops" > $O/pytest.log 2>&1 || { echo "tests failed"; grep -v "^E  *$" $O/pytest.log | tail -80; exit 1; }
tail -8 $O/pytest.log
