set -o pipefail
# Round 4: recursive doubling over host windows keeps every barrier when a copy fails; user-op tests
O=gpurun_out/r04ua
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_collectives_mp.py -k "user or strided or random" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -n 3 $O/pytest.log
