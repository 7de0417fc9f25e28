set -o pipefail
# Re-entry check: GPU tests, bench line + rocprof stats (tools/gpu_check.sh),
# then the 2-rank shared-GPU bench line (N>1 code path on the 1-GPU box).
bash tools/gpu_check.sh r01g || exit 1
O=gpurun_out/r01g
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
