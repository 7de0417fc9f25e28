set -o pipefail
# Round 5, pass k: the 8-rank line with point-to-point copies on the copy engines
# (MV2AMD_P2P_KERNEL_COPY=0): is the user-op staging's all-to-all (18.5 ms per call at 8 shared
# ranks in r05j against 4.7 ms in r04w) slowed by 8 processes' copy kernels contending for the
# shared GPU's compute queues?
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
MV2AMD_P2P_KERNEL_COPY=0 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29608 bench.py --gpus 8 --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_torchrun8_k0.json 2> $O/bench_torchrun8_k0.err || { tail -30 $O/bench_torchrun8_k0.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r05k/bench_torchrun8_k0.json", "profiles/r05j/bench_torchrun8.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["extra"]["pt2pt_bw_16MiB_x8"]["GBps"])
    for k, v in d["extra"].items():
        if k.startswith("allreduce_user"): print("  ", k, v["ms"], v["phases_ms_rank0"])
    sw = d["extra"]["osu_sweep"]
    print("  lat", sw["osu_latency_us"][::3], "bw", sw["osu_bw_GBps"][::3])
PY
