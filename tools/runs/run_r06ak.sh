#!/bin/bash
set -o pipefail
# Round 6, pass ak: a collective one rank never enters -- the other's device wait runs out after 2 s and
# is reported (the waiting launch, the slot re-read from memory), both ranks finalize
O=gpurun_out/r06ak
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v -m gpu --timeout 150 --timeout-method thread "tests/test_gpu_collectives_mp.py::test_absent_peer_is_reported_not_hung" "tests/test_gpu_collectives_mp.py::test_collectives_multiprocess[2-default]" > $O/pytest.log 2>&1 || { echo failed; tail -50 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
