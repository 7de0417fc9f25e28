#!/bin/bash
set -o pipefail
# Round 6, pass h: the 8-byte MPI_Reduce_local through the library's own HSA queue (runtime/aql.cpp)
# against the HIP launch (MV2AMD_AQL=0) and the platform floor; the Reduce_local GPU tests (every
# (op, type) pair at counts 1 and 7 now takes the queue); the N = 1 line (kernel time of the 256 MiB
# call after the completion word's 64-bit XCD-checked counters)
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 tools/diag/rl_lat lib 5000 | tee $O/lib_aql.jsonl || exit 1
MV2AMD_AQL=0 timeout -k 10 60 tools/diag/rl_lat lib 5000 | tee $O/lib_hip.jsonl || exit 1
timeout -k 10 60 tools/diag/rl_lat floor 5000 | tee $O/floor.jsonl || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_reduce_local.py > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc = 0 ] || { grep -B5 -A30 "Error\|FAIL" $O/pytest.log | head -80; exit 1; }
timeout -k 10 300 python3 bench.py --cpu-seconds 0 > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
print('N=1', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['extra']['reduce_local_8B_latency_us'], d['extra']['completion_word'])"
