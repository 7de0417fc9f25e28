set -o pipefail
# Round 3, pass ac: point-to-point + nonblocking collectives above 8 ranks (12 as 3x4, 10 as 10x1)
O=gpurun_out/r03ac
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_p2p_mp.py -k "12-4 or 10-1" > $O/pytest.log 2>&1 || { echo "tests failed"; grep -n "rank\|Error\|assert" $O/pytest.log | tail -60; exit 1; }
tail -3 $O/pytest.log
