set -o pipefail
# Round 3, pass o: operands above 4 GiB (2 ranks sharing the GPU).
O=gpurun_out/r03o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v -m gpu --timeout 600 --timeout-method thread tests/test_gpu_collectives_mp.py -k above_4gib > $O/pytest_huge.log 2>&1 || { echo "huge test failed"; tail -80 $O/pytest_huge.log; exit 1; }
tail -3 $O/pytest_huge.log
