set -o pipefail
# Round 5, pass j: the N > 1 line at 8 ranks (all on the one GPU: a rehearsal of the driver's N = 8
# path -- 8-rank orders, sweeps with their child job, point-to-point rows, user-op lines)
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29608 bench.py --gpus 8 --steps 10 --warmup 3 > $O/bench_torchrun8.json 2> $O/bench_torchrun8.err || { tail -30 $O/bench_torchrun8.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05j/bench_torchrun8.json").read().strip().splitlines()[-1])
sw = d["extra"].get("osu_sweep", {})
print(8, d["value"], d["config"]["latency_8B_us"], d["config"].get("latency_8B_us_python_loop"), sw.get("seconds"), sw.get("all_valid"), sw.get("error"),
      d["extra"]["pt2pt_bw_16MiB_x8"]["GBps"], d["cpu_baseline"]["value"], d["config"]["correct"])
for c in ("allreduce", "reduce_scatter", "allgather", "bcast"):
    print(" ", c, [(r[0], r[1], r[2]) for r in sw.get(c, [])][::2])
print({k: v for k, v in d["extra"].items() if isinstance(v, dict) and "busbw_GBps" in v})
PY
