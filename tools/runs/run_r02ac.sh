set -o pipefail
O=gpurun_out/r02ac
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
MV2AMD_PIPE_AUTOTUNE=1 timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share_autotune.json 2> $O/bench_2share_autotune.err || { tail -20 $O/bench_2share_autotune.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_2share_autotune.json'));print(d['value'], d['config']['latency_8B_us'], d['config']['pipe_tiling'], d['extra']['reduce_scatter_f32_sum'], d['extra']['allgather_char'], d['extra']['bcast_char'], d['extra']['allreduce_maxloc_double_int'])"
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_2share.json'));print(d['value'], d['config']['pipe_tiling'])"
MV2AMD_PIPE_AUTOTUNE=1 timeout -k 10 300 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 290 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lat-iters 200 > $O/bench_8share_autotune.json 2> $O/bench_8share_autotune.err || { tail -20 $O/bench_8share_autotune.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_8share_autotune.json'));print(d['value'], d['config']['pipe_tiling'])"
