set -o pipefail
O=gpurun_out/r02ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives_mp.py -k "autotune" -x -v --timeout 200 --timeout-method thread > $O/pytest_autotune.log 2>&1 || { tail -40 $O/pytest_autotune.log; exit 1; }
tail -1 $O/pytest_autotune.log
MV2AMD_PIPE_AUTOTUNE=1 timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share_autotune.json 2> $O/bench_2share_autotune.err || { tail -20 $O/bench_2share_autotune.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_2share_autotune.json'));print(d['value'], d['config']['pipe_tiling'], d['extra']['reduce_scatter_f32_sum'], d['extra']['allgather_char'])"
MV2AMD_PIPE_AUTOTUNE=1 timeout -k 10 300 python -m mvapich2_amd.mv2run -n 4 --share-gpu --timeout 290 python -u bench.py --gpus 4 --steps 5 --warmup 2 --lat-iters 200 > $O/bench_4share_autotune.json 2> $O/bench_4share_autotune.err || { tail -20 $O/bench_4share_autotune.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_4share_autotune.json'));print(d['value'], d['config']['pipe_tiling'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
