set -o pipefail
# Round 5, pass d: the new GPU tests (self-test count, late hardware-queue report), the whole suite,
# the N = 1 line (host baseline with its STREAM bound) and the 2-rank line (sweep child with the
# parent's tuning)
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread tests/test_gpu_collectives_mp.py -k "hw_queue or autotune" > $O/pytest_new.log 2>&1 || { tail -60 $O/pytest_new.log; exit 1; }
tail -4 $O/pytest_new.log
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05d/bench_n1.json").read().strip().splitlines()[-1])
print("N=1", d["value"], d["roofline"]["frac"], json.dumps(d["extra"]["cpu_host_allreduce_8rank"])[:900])
d = json.loads(open("gpurun_out/r05d/bench_torchrun2.json").read().strip().splitlines()[-1])
sw = d["extra"].get("osu_sweep", {})
print("N=2", d["value"], sw.get("seconds"), sw.get("all_valid"), [r[:3] for r in sw.get("allreduce", [])][-3:])
PY
