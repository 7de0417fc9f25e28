set -o pipefail
# The driver's N>1 launch line (torch.distributed.run), rehearsed with 2 ranks on the one GPU.
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
tail -1 $O/bench_torchrun2.json | cut -c1-600
