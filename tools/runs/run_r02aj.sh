set -o pipefail
O=gpurun_out/r02aj
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['frac'], d['extra']['MPI_Pack/Unpack MPI_Type_vector(8Mi,4,8,MPI_FLOAT)'])"
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 3 --share-gpu --timeout 290 python -u bench.py --gpus 3 --steps 5 --warmup 2 --lat-iters 300 > $O/bench_3share.json 2> $O/bench_3share.err || { tail -20 $O/bench_3share.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_3share.json'));print(d['value'], d['config']['correct'], d['config']['pipe_tiling']['grid'], d['extra']['allgather_char'])"
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 290 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lat-iters 300 > $O/bench_8share.json 2> $O/bench_8share.err || { tail -20 $O/bench_8share.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_8share.json'));print(d['value'], d['config']['correct'])"
