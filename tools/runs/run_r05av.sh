set -o pipefail
# Round 5, pass av: the soak list with the 8 = 2 x 4 emulated-node case
O=gpurun_out/r05av
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_collectives_mp.py::test_soak_thousands_of_calls" > $O/pytest.log 2>&1; rc=$?; tail -14 $O/pytest.log; exit $rc
