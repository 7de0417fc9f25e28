set -o pipefail
# Re-entry check after container re-creation: GPU tests (incl. derived-datatype
# pack path), bench line + rocprof stats, 2-rank shared-GPU bench line.
bash tools/gpu_check.sh r01h || exit 1
O=gpurun_out/r01h
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
