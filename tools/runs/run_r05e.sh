set -o pipefail
# Round 5, pass e: the 2-rank line with the point-to-point rows in its OSU sweep
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05e/bench_torchrun2.json").read().strip().splitlines()[-1])
sw = d["extra"].get("osu_sweep", {})
print("N=2", d["value"], sw.get("seconds"), sw.get("all_valid"), sw.get("error"))
print(sw.get("osu_latency_us"))
print(sw.get("osu_bw_GBps"))
PY
