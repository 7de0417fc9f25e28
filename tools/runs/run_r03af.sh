set -o pipefail
# Round 3, pass af: two-level table entries across nodes incl. 8 ranks as 4x2 (the numproc 8 entry's
# pt2pt_rs intra step at 64-127 B with the shortcuts off)
O=gpurun_out/r03af
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_multinode_mp.py -k "table_entries" > $O/pytest.log 2>&1 || { echo "tests failed"; grep -v "^E  *$" $O/pytest.log | tail -60; exit 1; }
tail -6 $O/pytest.log
