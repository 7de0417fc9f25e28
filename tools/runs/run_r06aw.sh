#!/bin/bash
set -o pipefail
# Round 6, pass aw: with the atomic flag polls -- the N > 1 line at 8 shared ranks (the driver's
# scaling-run shape) and the whole -m gpu suite twice more
O=gpurun_out/r06aw
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29638 bench.py --gpus 8 > $O/bench_torchrun8.json 2> $O/bench_torchrun8.err || { tail -30 $O/bench_torchrun8.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_torchrun8.json').read().strip().splitlines()[-1]); sw=d['extra'].get('osu_sweep', {})
print('N=8', d['value'], d['config']['latency_8B_us'], sw.get('all_valid'), d['config'].get('timed_calls_verified'), d['config'].get('correct'))"
for k in 1 2; do
  timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest$k.log 2>&1; rc=$?
  tail -1 $O/pytest$k.log
  grep -n "FAILED\|the waited slot now\|waited for epoch" $O/pytest$k.log | cut -c1-300 | head -20
  [ $rc -eq 0 ] || exit $rc
done
