set -o pipefail
# Round 5, pass l: the whole suite with the point-to-point copy policy (kernels at <= 2 ranks per
# GPU); the 4- and 8-rank lines (copy engines) against r05i / r05j
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29604 bench.py --gpus 4 --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_torchrun4.json 2> $O/bench_torchrun4.err || { tail -30 $O/bench_torchrun4.err; exit 1; }
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29608 bench.py --gpus 8 --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_torchrun8.json 2> $O/bench_torchrun8.err || { tail -30 $O/bench_torchrun8.err; exit 1; }
python3 - <<'PY'
import json
for n in (4, 8):
    d = json.loads(open(f"gpurun_out/r05l/bench_torchrun{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["config"]["latency_8B_us"], d["extra"]["pt2pt_bw_16MiB_x8"]["GBps"], d["extra"]["osu_sweep"]["all_valid"])
    for k, v in d["extra"].items():
        if k.startswith("allreduce_user"): print("  ", k, v["ms"], v["phases_ms_rank0"])
PY
