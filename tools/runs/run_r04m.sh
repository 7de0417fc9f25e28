set -o pipefail
# Round 4, pass m: user-op recursive doubling with its exchanges through host windows — the
# collectives, the MPICH collective suite (device and host operands) and the bench's user-op lines
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_collectives_mp.py tests/test_gpu_mpich_coll_suite.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -80 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29603 bench.py --gpus 8 --steps 5 --warmup 2 > $O/bench_torchrun8.json 2> $O/bench_torchrun8.err || { tail -30 $O/bench_torchrun8.err; exit 1; }
python3 -c "
import json
for f in ('$O/bench_torchrun2.json', '$O/bench_torchrun8.json'):
    d = json.load(open(f)); e = d['extra']
    print(f, d['value'], {k: v.get('ms') for k, v in e.items() if k.startswith('allreduce_user_op')})
"
