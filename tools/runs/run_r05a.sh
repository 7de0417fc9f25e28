set -o pipefail
# Round 5, pass a: smoke; the 2-rank line (MPI_Init's new self-test and its time split); the whole
# -m gpu suite on the cut fatbin; the N = 1 line; the RCCL comparator child at WORLD_SIZE = 1
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
grep "MPI_Init" $O/bench_torchrun2.err | head -2
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
MV2AMD_INIT_REPORT=1 timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
grep "MPI_Init" $O/bench_n1.err | head -2
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29651 MV2AMD_RCCL_STEPS=10 timeout -k 10 240 python3 bench.py --rccl-child > $O/rccl_child_ws1.json 2> $O/rccl_child_ws1.err; echo "rccl child rc=$?"
cat $O/rccl_child_ws1.json
cut -c1-600 $O/bench_n1.json
