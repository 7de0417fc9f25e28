set -o pipefail
O=gpurun_out/r02q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 3 --share-gpu --timeout 230 python -u bench.py --gpus 3 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_3share.json 2> $O/bench_3share.err || { tail -20 $O/bench_3share.err; exit 1; }
cat $O/bench_3share.json
