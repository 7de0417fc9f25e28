set -o pipefail
# Round 3, pass r: the lingering one-shot kernel — its own test, the multiprocess collectives,
# then the 2-rank bench (8-byte latency) with the window on and off.
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_collectives_mp.py -k "lingering" > $O/pytest_linger.log 2>&1 || { echo "linger tests failed"; tail -100 $O/pytest_linger.log; exit 1; }
tail -3 $O/pytest_linger.log
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_collectives_mp.py tests/test_gpu_p2p_mp.py > $O/pytest_coll.log 2>&1 || { echo "collective tests failed"; tail -100 $O/pytest_coll.log; exit 1; }
tail -3 $O/pytest_coll.log
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 290 python -u bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
MV2AMD_LINGER_US=0 timeout -k 10 300 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 290 python -u bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_2share_nolinger.json 2> $O/bench_2share_nolinger.err || { tail -20 $O/bench_2share_nolinger.err; exit 1; }
python3 -c "
import json
for f in ['$O/bench_2share.json','$O/bench_2share_nolinger.json']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); c=d['config']
    print(f, d['value'], c['latency_8B_us'], c['latency_8B_max_over_ranks_us'], c['latency_8B_kernel_us'], c['correct'])
"
