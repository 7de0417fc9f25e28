#!/bin/bash
set -o pipefail
# Round 6, pass f: the new tests (completion-word counters; more than 8 processes per GPU refused
# at MPI_Init, incl. the restored 12 = 3 x 4 random sequence), the self-test after its buffer fix
# (autotune test asserts its 43 calls), then one 12 = 3 x 4 ring soak, which must now end in the
# explicit refusal on every rank
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_reduce_local.py::test_completion_word_fallbacks_are_counted" \
  "tests/test_gpu_collectives_mp.py::test_more_than_8_processes_per_gpu_are_refused" \
  "tests/test_gpu_collectives_mp.py::test_random_sequence_across_nodes" \
  "tests/test_gpu_collectives_mp.py::test_pipe_autotune_agrees_and_keeps_results" > $O/pytest.log 2>&1
rc=$?; tail -25 $O/pytest.log; [ $rc = 0 ] || exit $rc
DIAG_DETAIL=2 DIAG_CHECK_SB=1 timeout -k 10 300 python -u tools/ringsoak_diag.py 12 4 400 32 $O/soak12x4 > $O/soak12x4.json 2> $O/soak12x4.err
echo "soak rc $?"; python3 -c "
import json; d=json.load(open('$O/soak12x4.json')); print('12x4 soak: rcs', d['rcs'], 'refused', d['refused'], 'results', [len(r) for r in d['per_rank']])" | tee $O/summary.txt
