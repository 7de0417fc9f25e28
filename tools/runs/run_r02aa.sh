set -o pipefail
# autotune test + shared-GPU bench lines with the autotune forced; PMC traffic of the new pack kernel
O=gpurun_out/r02aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_collectives_mp.py -k "autotune" -x -v --timeout 200 --timeout-method thread > $O/pytest_autotune.log 2>&1 || { tail -40 $O/pytest_autotune.log; exit 1; }
tail -3 $O/pytest_autotune.log
MV2AMD_PIPE_AUTOTUNE=1 timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share_autotune.json 2> $O/bench_2share_autotune.err || { tail -20 $O/bench_2share_autotune.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_2share_autotune.json'));print(d['value'], d['config']['pipe_tiling'])"
pmc() {  # name counter cmd...
    local name=$1 c=$2; shift 2
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/${name}_$c -o p -- "$@" > $O/${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; tail -5 $O/${name}_$c.log; return 1; }
    find $O/${name}_$c -name '*counter_collection.csv' > $O/${name}_$c.path
}
summ() {  # name match algbytes
    python tools/pmc_summary.py "$(cat $O/${1}_FETCH_SIZE.path)" "$(cat $O/${1}_WRITE_SIZE.path)" "$2" $O/pmc_$1.json $3 && cat $O/pmc_$1.json
}
for mode in pack unpack; do
    for c in FETCH_SIZE WRITE_SIZE; do PMC_MODE=$mode pmc $mode $c python3 tools/pmc_pack.py || exit 1; done
    summ $mode "k_pack" 268435456 || exit 1
done
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 290 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lat-iters 200 > $O/bench_8share.json 2> $O/bench_8share.err || { tail -20 $O/bench_8share.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_8share.json'));print(d['value'], d['config']['latency_8B_us'], d['config']['pipe_tiling'])"
