set -o pipefail
# Round 4, final tree after the one-shot reduce-scatter: smoke, the N = 1 line with rocprofv3 kernel statistics, 2 / 4-rank rehearsals (the whole -m gpu suite ran in r04rs on this build)
O=gpurun_out/r04fin
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29632 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29634 bench.py --gpus 4 --steps 5 --warmup 2 > $O/bench_torchrun4.json 2> $O/bench_torchrun4.err || { tail -30 $O/bench_torchrun4.err; exit 1; }
cut -c1-220 $O/bench_n1.json $O/bench_torchrun2.json $O/bench_torchrun4.json
