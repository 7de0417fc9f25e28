set -o pipefail
# Round 3, pass ag: the driver's N=4 and N=8 launch lines rehearsed with every rank on the one GPU
# (torchrun, one process per rank; no xGMI byte moves, so the numbers are shared-GPU lines)
O=gpurun_out/r03ag
mkdir -p $O
export TMPDIR=/tmp
for N in 4 8; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N --steps 5 --warmup 2 > $O/bench_torchrun$N.json 2> $O/bench_torchrun$N.err || { tail -30 $O/bench_torchrun$N.err; exit 1; }
  tail -1 $O/bench_torchrun$N.json | cut -c1-700
done
