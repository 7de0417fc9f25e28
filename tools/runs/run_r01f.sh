set -o pipefail
bash tools/gpu_check.sh r01f || exit 1
O=gpurun_out/r01f
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
