#!/bin/bash
set -o pipefail
# Round 6, pass ap: flag polls as never-writing atomics -- the 2-rank line (pipelined 256 MiB rounds
# poll too) and the whole -m gpu suite three more times
O=gpurun_out/r06ap
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_torchrun2.json').read().strip().splitlines()[-1]); sw=d['extra']['osu_sweep']
print('N=2', d['value'], d['config']['latency_8B_us'], sw['all_valid'], d['config'].get('timed_calls_verified'))"
for k in 1 2 3; do
  timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest$k.log 2>&1; rc=$?
  tail -1 $O/pytest$k.log
  grep -n "FAILED\|the waited slot now\|waited for epoch" $O/pytest$k.log | cut -c1-300 | head -20
  [ $rc -eq 0 ] || exit $rc
done
