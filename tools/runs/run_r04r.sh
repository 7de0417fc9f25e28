set -o pipefail
# Round 4, pass r: the user-op lines' phase breakdown (stage / fetch / eval / deliver) at 2 and 8 ranks
O=gpurun_out/r04r
mkdir -p $O
export TMPDIR=/tmp
for nr in 2 8; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $nr --master-addr 127.0.0.1 --master-port 2962$nr bench.py --gpus $nr --steps 5 --warmup 2 --cpu-seconds 0 --rccl 0 > $O/bench_torchrun$nr.json 2> $O/bench_torchrun$nr.err || { tail -30 $O/bench_torchrun$nr.err; exit 1; }
done
python3 -c "
import json
for nr in (2, 8):
    d = json.load(open('$O/bench_torchrun%d.json' % nr)); e = d['extra']
    for k, v in e.items():
        if k.startswith('allreduce_user_op'): print(nr, k, v['ms'], v['phases_ms_rank0'])
"
