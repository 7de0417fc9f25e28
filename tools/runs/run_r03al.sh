set -o pipefail
# Round 3, pass al: the round-end tree: the whole -m gpu suite, N=1 bench + kernel stats,
# stats, the driver's N=2 torchrun launch line on the shared GPU.
O=gpurun_out/r03al
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; grep -v "^E  *$" $O/pytest.log | tail -80; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
cut -c1-400 $O/bench_n1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec head -6 {} \;
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
tail -1 $O/bench_torchrun2.json | cut -c1-400
