set -o pipefail
# Round 5, pass bd: the N > 1 line at 4 and 8 ranks on the final library (a rehearsal of the driver's
# scaling run, every rank sharing the one GPU), and OSU allreduce 4 B - 4 KiB at 8 shared ranks
O=gpurun_out/r05bd
mkdir -p $O
export TMPDIR=/tmp
for n in 4 8; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2961$n bench.py --gpus $n > $O/bench_torchrun$n.json 2> $O/bench_torchrun$n.err || { tail -30 $O/bench_torchrun$n.err; exit 1; }
done
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 190 tools/osu/osu_coll -c allreduce -m 4:4096 -i 2000 -x 200 -v > $O/ar_8.txt 2>&1 || { tail -20 $O/ar_8.txt; exit 1; }
grep -v "^#\|MPI_Init" $O/ar_8.txt | head -12
python3 - <<'PY'
import json
for n in (4, 8):
    d = json.loads(open(f"gpurun_out/r05bd/bench_torchrun{n}.json").read().strip().splitlines()[-1])
    sw = d["extra"]["osu_sweep"]
    print(f"N={n}", d["value"], d["unit"], d["config"]["latency_8B_us"], sw["all_valid"], d["roofline"].get("frac"), d["cpu_baseline"]["value"])
    print(" ", [(r[0], r[1], r[2]) for r in sw["allreduce"]][::3])
PY
