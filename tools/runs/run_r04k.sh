set -o pipefail
# Round 4, pass k: the protocol under the full-release fallback and non-default tilings
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 280 --timeout-method thread tests/test_gpu_collectives_mp.py -k "test_release_and_tiling_variants" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
