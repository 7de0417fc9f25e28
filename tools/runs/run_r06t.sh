#!/bin/bash
set -o pipefail
# Round 6, pass t: the one-shot allreduce through the library's HSA queue (aql_launch) at 2 ranks on
# the one GPU: the 2-rank collective tests and soaks, then the 2-rank line (8-byte OSU latency; the
# queue's launches counted) against MV2AMD_AQL=0
O=gpurun_out/r06t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_collectives_mp.py -k "2 or soak" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -B5 -A40 "Error\|FAIL" $O/pytest.log | head -120; exit 1; }
for aql in 1 0; do
  MV2AMD_AQL=$aql timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2961$aql bench.py --gpus 2 --rccl 0 > $O/bench2_aql$aql.json 2> $O/bench2_aql$aql.err || { tail -30 $O/bench2_aql$aql.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench2_aql$aql.json').read().strip().splitlines()[-1]); sw=d['extra']['osu_sweep']
print('aql=$aql', d['value'], d['config']['latency_8B_us'], d['config']['latency_8B_us_python_loop'], sw['all_valid'], [(r[0], r[1]) for r in sw['allreduce']][:4], d['config'].get('timed_calls_verified'))"
done
