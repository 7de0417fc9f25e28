set -o pipefail
# End-of-round measurement pass (second, after the autotune and multi-node additions): GPU suite, N=1 bench + rocprof kernel stats, PMC traffic of the
# hot kernels (separate FETCH_SIZE / WRITE_SIZE passes), shared-GPU bench lines at 2/3/8 ranks.
O=gpurun_out/r02final2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
pmc() {  # name counter cmd...
    local name=$1 c=$2; shift 2
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/${name}_$c -o p -- "$@" > $O/${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; tail -5 $O/${name}_$c.log; return 1; }
    find $O/${name}_$c -name '*counter_collection.csv' > $O/${name}_$c.path
}
summ() {  # name match algbytes
    python tools/pmc_summary.py "$(cat $O/${1}_FETCH_SIZE.path)" "$(cat $O/${1}_WRITE_SIZE.path)" "$2" $O/pmc_$1.json $3 && cat $O/pmc_$1.json
}
for c in FETCH_SIZE WRITE_SIZE; do pmc rl $c python3 tools/pmc_reduce_local.py || exit 1; done
summ rl "k_reduce_local<mv2::R<2, 8, void>, 2>" 805306368 || exit 1
for mode in pack unpack; do
    for c in FETCH_SIZE WRITE_SIZE; do PMC_MODE=$mode pmc $mode $c python3 tools/pmc_pack.py || exit 1; done
    summ $mode "k_pack" 268435456 || exit 1
done
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 500 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
MV2AMD_PIPE_AUTOTUNE=1 timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 500 > $O/bench_2share_autotune.json 2> $O/bench_2share_autotune.err || { tail -20 $O/bench_2share_autotune.err; exit 1; }
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 3 --share-gpu --timeout 290 python -u bench.py --gpus 3 --steps 5 --warmup 2 --lat-iters 300 > $O/bench_3share.json 2> $O/bench_3share.err || { tail -20 $O/bench_3share.err; exit 1; }
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 290 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lat-iters 300 > $O/bench_8share.json 2> $O/bench_8share.err || { tail -20 $O/bench_8share.err; exit 1; }
for f in bench bench_2share bench_2share_autotune bench_3share bench_8share; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['roofline'].get('frac'), d['config'].get('latency_8B_us'))"; done
