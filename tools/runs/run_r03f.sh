set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_mpich_datatype_suite.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -6 $O/pytest.log
timeout -k 10 100 ./tests/mpich_datatype/dt_suite device > $O/dt_device.txt 2>&1; cat $O/dt_device.txt
