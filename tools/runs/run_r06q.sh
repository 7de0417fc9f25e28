#!/bin/bash
set -o pipefail
# Round 6, pass q: the HSA-queue path with the agent-scope acquire of a one-rank job: C-loop latency,
# the Reduce_local tests, the N = 1 line's 8-byte figures
O=gpurun_out/r06q
mkdir -p $O
export TMPDIR=/tmp
MV2AMD_HOST_PROFILE=200 timeout -k 10 60 tools/diag/rl_lat lib 5000 2>&1 | tee $O/lib.txt || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_reduce_local.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -B5 -A40 "Error\|FAIL" $O/pytest.log | head -100; exit 1; }
timeout -k 10 300 python3 bench.py --cpu-seconds 0 > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
print('N=1', d['value'], d['roofline']['frac'], d['extra']['reduce_local_8B_latency_us'])"
