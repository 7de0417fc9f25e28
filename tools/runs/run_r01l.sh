set -o pipefail
# 2-rank shared-GPU bench: lazy P2P stream + plain stores to own buffers in the pipe kernels
O=gpurun_out/r01l
mkdir -p $O
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 --rccl 0 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives_mp.py tests/test_gpu_p2p_mp.py -x -q --timeout 150 --timeout-method thread > $O/mp.log 2>&1; tail -3 $O/mp.log
