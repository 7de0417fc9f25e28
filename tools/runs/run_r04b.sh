set -o pipefail
# Round 4, pass b: k_pipe PMC traffic at 2 / 4 / 8 ranks sharing the GPU (the configuration recorded
# in each summary, bench.py pipe_traffic_for), then the 4- and 8-rank torchrun rehearsals of the
# N > 1 bench line (cpu_baseline on rank 0 after MPI_Finalize; MPI_Init's report on stderr).
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp
pmc() {  # name counter cmd...
    local name=$1 c=$2; shift 2
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${name}_$c -o p -- "$@" > $O/${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; tail -5 $O/${name}_$c.log; return 1; }
    find $O/${name}_$c -name '*counter_collection.csv' > $O/${name}_$c.path
}
pipe_pass() {  # n counter
    local n=$1 c=$2 J=p$RANDOM$RANDOM pids=()
    for r in $(seq 1 $((n - 1))); do
        RANK=$r WORLD_SIZE=$n LOCAL_RANK=$r LOCAL_WORLD_SIZE=$n MV2AMD_JOBID=$J MV2AMD_TIMEOUT_S=60 MV2AMD_DEVICE=0 timeout -k 5 110 python3 tools/pmc_pipe.py > $O/pipe${n}_r${r}_$c.log 2>&1 &
        pids+=($!)
    done
    RANK=0 WORLD_SIZE=$n LOCAL_RANK=0 LOCAL_WORLD_SIZE=$n MV2AMD_JOBID=$J MV2AMD_TIMEOUT_S=60 MV2AMD_DEVICE=0 PMC_CONFIG_OUT=$O/pipe${n}_cfg.json pmc pipe$n $c python3 tools/pmc_pipe.py
    local r0=$? bad=0
    for p in "${pids[@]}"; do wait $p || bad=1; done
    [ $r0 = 0 ] && [ $bad = 0 ] || { echo "pipe pass n=$n $c failed ($r0 $bad)"; tail -5 $O/pipe${n}_r1_$c.log; return 1; }
}
for n in 2 4 8; do
    pipe_pass $n FETCH_SIZE || exit 1
    pipe_pass $n WRITE_SIZE || exit 1
    alg=$(python3 -c "n=$n; S=64<<20; print(int(2*S*(1+2*(n-1)/n)))")
    python3 tools/pmc_summary.py "$(cat $O/pipe${n}_FETCH_SIZE.path)" "$(cat $O/pipe${n}_WRITE_SIZE.path)" "k_pipe<mv2::R<2, 8" $O/pmc_pipe_allreduce_${n}rank_r04b.json $alg 6 $O/pipe${n}_cfg.json > /dev/null || exit 1
    cp $O/pmc_pipe_allreduce_${n}rank_r04b.json profiles/
done
for n in 4 8; do
    timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 > $O/bench_torchrun$n.json 2> $O/bench_torchrun$n.err || { tail -30 $O/bench_torchrun$n.err; exit 1; }
    grep "MPI_Init:" $O/bench_torchrun$n.err || true
done
echo r04b done
