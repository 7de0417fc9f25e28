set -o pipefail
# Round 5, pass aw: the jobs-above-8-ranks tests moved to at most 8 processes
# (MV2AMD_MN_PROG_MAX=4 for the schedules; 8 x 1 and 2 x 4 point-to-point)
O=gpurun_out/r05aw
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_multinode_mp.py::test_more_than_eight_ranks_across_nodes" \
  "tests/test_gpu_multinode_mp.py::test_user_ops_across_nodes" \
  "tests/test_gpu_p2p_mp.py" > $O/pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -25; exit $rc
