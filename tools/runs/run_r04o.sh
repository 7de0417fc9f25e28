set -o pipefail
# Round 4, pass o: the RD exchange from 4 ranks on (MV2AMD_UOP_EXCHANGE), tests and A/B bench lines
O=gpurun_out/r04o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_collectives_mp.py tests/test_gpu_mpich_coll_suite.py -k "strided_vector or collectives_multiprocess or coll_suite" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -80 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for nr in 4 8; do
  for x in 0 -1; do
    MV2AMD_UOP_EXCHANGE=$x timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $nr --master-addr 127.0.0.1 --master-port 2961$nr bench.py --gpus $nr --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_torchrun${nr}_x$x.json 2> $O/bench_torchrun${nr}_x$x.err || { tail -30 $O/bench_torchrun${nr}_x$x.err; exit 1; }
  done
done
python3 -c "
import json, glob
for f in sorted(glob.glob('$O/bench_torchrun*.json')):
    d = json.load(open(f)); e = d['extra']
    print(f, d['value'], {k: v.get('ms') for k, v in e.items() if k.startswith('allreduce_user_op')})
"
