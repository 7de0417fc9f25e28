set -o pipefail
# Round 3, pass e: the reference's restated MPICH collective tests (tests/mpich_coll).
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_mpich_coll_suite.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 4 --share-gpu --timeout 180 ./tests/mpich_coll/coll_suite device > $O/suite_dev4.txt 2>&1 || { cat $O/suite_dev4.txt | tail -30; exit 1; }
cat $O/suite_dev4.txt
