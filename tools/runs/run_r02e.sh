set -o pipefail
# Round-2 measurement pass: PMC traffic of the current Reduce_local kernel, of the
# pack / unpack kernels (configs[4] vector type) and of the pipelined allreduce
# kernel (2 ranks on one GPU: rank 0 under rocprofv3, rank 1 plain), then the
# 2- and 8-rank shared-GPU bench lines.
O=gpurun_out/r02e
mkdir -p $O
export TMPDIR=/tmp
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
# pipelined allreduce, 64 MiB fp32 SUM, 2 ranks sharing the GPU
pipe_pass() {  # counter
    local c=$1 J=p$RANDOM$RANDOM
    RANK=1 WORLD_SIZE=2 LOCAL_RANK=1 LOCAL_WORLD_SIZE=2 MV2AMD_JOBID=$J MV2AMD_TIMEOUT_S=40 timeout -k 5 80 python3 tools/pmc_pipe.py > $O/pipe_r1_$c.log 2>&1 &
    local p1=$!
    RANK=0 WORLD_SIZE=2 LOCAL_RANK=0 LOCAL_WORLD_SIZE=2 MV2AMD_JOBID=$J MV2AMD_TIMEOUT_S=40 pmc pipe $c python3 tools/pmc_pipe.py
    local r0=$?
    wait $p1
    local r1=$?
    [ $r0 = 0 ] && [ $r1 = 0 ] || { echo "pipe pass $c failed ($r0 $r1)"; tail -5 $O/pipe_r1_$c.log; return 1; }
}
pipe_pass FETCH_SIZE || exit 1
pipe_pass WRITE_SIZE || exit 1
summ pipe "k_pipe" 268435456 || exit 1
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 290 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lat-iters 200 > $O/bench_8share.json 2> $O/bench_8share.err || { tail -20 $O/bench_8share.err; exit 1; }
cat $O/bench_8share.json
