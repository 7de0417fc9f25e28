set -o pipefail
# Round 5, pass c: the N > 1 line with its OSU sweeps (configs[2] / [3] through tools/osu/osu_coll)
# at 2 and 4 shared ranks; the RCCL comparator child with its size sweep at WORLD_SIZE = 1
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29604 bench.py --gpus 4 --steps 10 --warmup 3 > $O/bench_torchrun4.json 2> $O/bench_torchrun4.err || { tail -30 $O/bench_torchrun4.err; exit 1; }
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29651 MV2AMD_RCCL_STEPS=10 timeout -k 10 240 python3 bench.py --rccl-child > $O/rccl_child_ws1.json 2> $O/rccl_child_ws1.err; echo "rccl child rc=$?"
tail -1 $O/rccl_child_ws1.json | cut -c1-400
python3 - <<'PY'
import json
for n in (2, 4):
    d = json.loads(open(f"gpurun_out/r05c/bench_torchrun{n}.json").read().strip().splitlines()[-1])
    sw = d["extra"].get("osu_sweep", {})
    print(n, d["value"], d["config"]["latency_8B_us"], d["cpu_baseline"] and d["cpu_baseline"].get("value"), "sweep s", sw.get("seconds"), "valid", sw.get("all_valid"), sw.get("error"))
    for c in ("allreduce", "reduce_scatter", "allgather", "bcast"):
        print(" ", c, [(r[0], r[1], r[2]) for r in sw.get(c, [])][::2])
PY
