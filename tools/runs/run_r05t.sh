set -o pipefail
# Round 5, pass t: the soak under every protocol setting a node may adopt (full release, small
# pipeline rounds, copy-engine point-to-point, two emulated nodes)
O=gpurun_out/r05t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread --durations=0 \
  tests/test_gpu_collectives_mp.py -k "soak" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -14 $O/pytest.log
