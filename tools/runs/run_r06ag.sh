#!/bin/bash
set -o pipefail
# Round 6, pass ag: the collectives suite at 2 and 3 ranks with the settings of a rank that has its
# GPU to itself (full grids, MPI_Init's probes and 1 MiB one-shot slots, copy-kernel point-to-point)
O=gpurun_out/r06ag
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread "tests/test_gpu_collectives_mp.py::test_collectives_multiprocess[2-full]" "tests/test_gpu_collectives_mp.py::test_collectives_multiprocess[3-full]" > $O/pytest.log 2>&1 || { echo failed; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
