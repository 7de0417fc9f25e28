set -o pipefail
# Round 4, final pass on the committed tree (point-to-point back at four chunk slots): smoke, the p2p tests, the N = 1 line and 2 / 4-rank rehearsals
O=gpurun_out/r04final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
timeout -k 10 700 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_p2p_mp.py > $O/pytest_p2p.log 2>&1 || { echo "tests failed"; tail -60 $O/pytest_p2p.log; exit 1; }
tail -n 2 $O/pytest_p2p.log
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 4 --steps 5 --warmup 2 > $O/bench_torchrun4.json 2> $O/bench_torchrun4.err || { tail -30 $O/bench_torchrun4.err; exit 1; }
cut -c1-300 $O/bench_n1.json $O/bench_torchrun2.json $O/bench_torchrun4.json
