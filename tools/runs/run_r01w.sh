set -o pipefail
# Final tree of the round: GPU tests, N=1 bench + rocprof kernel stats, 2-rank and 8-rank shared-GPU bench lines.
bash tools/gpu_check.sh r01w || exit 1
O=gpurun_out/r01w
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
timeout -k 10 280 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 270 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lat-iters 100 --rccl 0 > $O/bench_8share.json 2> $O/bench_8share.err || { tail -20 $O/bench_8share.err; exit 1; }
cat $O/bench_8share.json
