set -o pipefail
# Round 3, pass p: the 2-rank user-op lines again (host-bound; r03n looked slow), via mv2run and torchrun.
O=gpurun_out/r03p
mkdir -p $O
nproc > $O/nproc.txt; uptime >> $O/nproc.txt
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 290 python -u bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
python3 -c "
import json
for f in ['$O/bench_2share.json','$O/bench_torchrun2.json']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); e=d['extra']
    print(f, d['value'], [(k, e[k]['ms']) for k in e if k.startswith('allreduce_user')])
"
cat $O/nproc.txt
