set -o pipefail
# Round 5, pass i: the tree as of now on the GPU: smoke; the N = 1 line; its rocprofv3 kernel
# statistics; the PMC HBM traffic of k_reduce_local for this binary (FETCH_SIZE and WRITE_SIZE in
# separate passes); the 2- and 4-rank rehearsals of the N > 1 line
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name '*kernel_stats*' | head -2
pmc() {  # name counter cmd...
    local name=$1 c=$2; shift 2
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/${name}_$c -o p -- "$@" > $O/${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; tail -5 $O/${name}_$c.log; return 1; }
    find $O/${name}_$c -name '*counter_collection.csv' > $O/${name}_$c.path
}
for c in FETCH_SIZE WRITE_SIZE; do pmc rl $c python3 tools/pmc_reduce_local.py || exit 1; done
python tools/pmc_summary.py "$(cat $O/rl_FETCH_SIZE.path)" "$(cat $O/rl_WRITE_SIZE.path)" "k_reduce_local<mv2::R<2, 8, void>, 2>" $O/pmc_reduce_local_r05i.json 805306368 6 && cat $O/pmc_reduce_local_r05i.json
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29604 bench.py --gpus 4 > $O/bench_torchrun4.json 2> $O/bench_torchrun4.err || { tail -30 $O/bench_torchrun4.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05i/bench_n1.json").read().strip().splitlines()[-1])
print("N=1", d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms"], d["cpu_baseline"]["value"])
for n in (2, 4):
    d = json.loads(open(f"gpurun_out/r05i/bench_torchrun{n}.json").read().strip().splitlines()[-1])
    sw = d["extra"].get("osu_sweep", {})
    print(n, d["value"], d["config"]["latency_8B_us"], d["config"].get("latency_8B_us_python_loop"), sw.get("all_valid"),
          d["extra"]["pt2pt_bw_16MiB_x8"]["GBps"], d["cpu_baseline"]["value"])
PY
