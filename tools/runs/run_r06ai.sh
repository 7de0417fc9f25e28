#!/bin/bash
set -o pipefail
# Round 6, pass ai: the N > 1 line at 4 and 8 ranks on the final tree on the one GPU (rehearsal of the driver's scaling
# run: every timed 256 MiB call verified, completion-word counts, release protocol, shared-GPU
# constants named), with the in-run OSU sweeps
O=gpurun_out/r06ai
mkdir -p $O
export TMPDIR=/tmp
for n in 4 8; do
  echo "== $n ranks $(date +%T)"
  timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2960$n bench.py --gpus $n > $O/bench_torchrun$n.json 2> $O/bench_torchrun$n.err || { tail -30 $O/bench_torchrun$n.err; exit 1; }
  python3 - $n <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads(open(f"gpurun_out/r06ai/bench_torchrun{n}.json").read().strip().splitlines()[-1])
sw = d["extra"].get("osu_sweep", {})
print(f"N={n}", d["value"], d["config"]["latency_8B_us"], sw.get("all_valid"), d["config"].get("timed_calls_verified"), d["config"].get("correct"),
      d["extra"].get("completion_word"), d["config"]["pipe_tiling"].get("release_protocol"), d["extra"].get("constants_tuned_on_shared_gpu"))
PY
done
