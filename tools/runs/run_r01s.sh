set -o pipefail
# Re-entry check after container re-creation: rebuilt tree, full GPU tests, bench + rocprof, 2-rank shared-GPU bench line.
# 2-rank shared-GPU bench line (now with the pt2pt bandwidth line).
bash tools/gpu_check.sh r01s || exit 1
O=gpurun_out/r01s
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
