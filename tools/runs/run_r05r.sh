set -o pipefail
# Round 5, pass r: the soak test (thousands of mixed calls at 2 / 4 / 8 shared ranks, every result
# checked) and the argument checks
O=gpurun_out/r05r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread --durations=0 \
  tests/test_gpu_collectives_mp.py -k "soak or argument_checks" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
