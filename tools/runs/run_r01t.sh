set -o pipefail
# Flat ring allreduce order from 2 MiB (MV2_ALLRED_USE_RING path) and the <= 1024 B two-level boundary: full GPU tests, bench + rocprof, 2-rank shared-GPU bench line.
bash tools/gpu_check.sh r01t || exit 1
O=gpurun_out/r01t
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
