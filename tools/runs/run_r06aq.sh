#!/bin/bash
set -o pipefail
# Round 6, pass aq: final validation with flag polls as never-writing atomics -- smoke, the whole -m gpu suite, the N = 1 line and
# its rocprofv3 kernel statistics, PMC traffic of the 256 MiB Reduce_local (FETCH_SIZE and WRITE_SIZE
# in separate passes), the 2-rank line with the OSU sweeps (every timed call verified)
O=gpurun_out/r06aq
mkdir -p $O
export TMPDIR=/tmp
ls /sys/class/kfd/kfd/proc > $O/kfd_procs_at_start.txt 2>&1 || true
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
cp $(find $O/prof -name '*kernel_stats*' | head -1) $O/rocprof_kernel_stats.csv && rm -rf $O/prof
pmc() {  # name counter cmd...
    local name=$1 c=$2; shift 2
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/${name}_$c -o p -- "$@" > $O/${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; tail -5 $O/${name}_$c.log; return 1; }
    find $O/${name}_$c -name '*counter_collection.csv' > $O/${name}_$c.path
}
for c in FETCH_SIZE WRITE_SIZE; do pmc rl $c python3 tools/pmc_reduce_local.py || exit 1; done
python tools/pmc_summary.py "$(cat $O/rl_FETCH_SIZE.path)" "$(cat $O/rl_WRITE_SIZE.path)" "k_reduce_local<mv2::R<2, 8, void>, 2>" $O/pmc_reduce_local_r06aq.json 805306368 6 && cat $O/pmc_reduce_local_r06aq.json
for c in FETCH_SIZE WRITE_SIZE; do rm -rf $O/rl_$c; done
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06aq/bench_n1.json").read().strip().splitlines()[-1])
print("N=1", d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms"], d["cpu_baseline"]["value"], d["extra"]["reduce_local_8B_latency_us"]["us"], d["extra"]["reduce_local_8B_latency_us"].get("python_loop_us"), d["extra"]["completion_word"], d["extra"]["cpu_host_allreduce_8rank"].get("l3_domains_used"), d["extra"]["cpu_host_allreduce_8rank"].get("latency_8B_us"))
d = json.loads(open("gpurun_out/r06aq/bench_torchrun2.json").read().strip().splitlines()[-1])
sw = d["extra"]["osu_sweep"]
print("N=2", d["value"], d["config"]["latency_8B_us"], sw["all_valid"], sw["osu_latency_us"][0], d["config"].get("timed_calls_verified"), d["extra"].get("completion_word"), d["config"]["pipe_tiling"].get("release_protocol"))
for c in ("allreduce", "reduce_scatter", "allgather", "bcast"):
    print(" ", c, [(r[0], r[1], r[2]) for r in sw[c]][::2])
PY
