set -o pipefail
# Round 4, pass u: the RD exchange copies the operand span and the result span directly (no host pack / unpack)
# eval_to_device): the user-op tests, then the phase breakdown at 2 and 8 ranks
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_collectives_mp.py tests/test_gpu_mpich_coll_suite.py tests/test_gpu_multinode_mp.py -k "strided_vector or collectives_multiprocess or coll_suite or user_ops" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -80 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for nr in 2 4 8; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $nr --master-addr 127.0.0.1 --master-port 2965$nr bench.py --gpus $nr --steps 5 --warmup 2 --cpu-seconds 0 --rccl 0 > $O/bench_torchrun$nr.json 2> $O/bench_torchrun$nr.err || { tail -30 $O/bench_torchrun$nr.err; exit 1; }
done
python3 -c "
import json
for nr in (2, 4, 8):
    d = json.load(open('$O/bench_torchrun%d.json' % nr)); e = d['extra']
    for k, v in e.items():
        if k.startswith('allreduce_user_op'): print(nr, k, v['ms'], v['phases_ms_rank0'])
"
