set -o pipefail
# Reduce_local variant sweep, then the full check (GPU tests, bench + rocprof)
# and the 2-rank shared-GPU bench line with the completion word + self-test.
mkdir -p gpurun_out/r01i
timeout -k 10 120 ./tools/rl_variants > gpurun_out/r01i/rl_variants.txt 2>&1 || exit 1
bash tools/gpu_check.sh r01i || exit 1
O=gpurun_out/r01i
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
