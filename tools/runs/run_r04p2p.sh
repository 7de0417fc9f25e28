set -o pipefail
# Round 4: point-to-point with 8 chunk slots per pair (was 4): the p2p tests and the osu_bw line
O=gpurun_out/r04p2p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_p2p_mp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2968$i bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 0 --rccl 0 > $O/bench_torchrun2_$i.json 2> $O/bench_torchrun2_$i.err || { tail -30 $O/bench_torchrun2_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_torchrun2_$i.json')); print(d['extra']['pt2pt_bw_16MiB_x8'])"
done
