#!/bin/bash
set -o pipefail
# Round 6, pass ae: the HSA-queue Reduce_local tests, the new system-scope acquire one included
O=gpurun_out/r06ae
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_reduce_local.py > $O/pytest.log 2>&1 || { echo "failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
