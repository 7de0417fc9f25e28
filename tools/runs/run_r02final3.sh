set -o pipefail
# PMC traffic of k_pipe (2 ranks, shared GPU) on the final tree (remote-store flavour + graph-lane
# sequence words added since r02au); separate FETCH_SIZE / WRITE_SIZE passes.
O=gpurun_out/r02final3
mkdir -p $O
export TMPDIR=/tmp
pmc() {  # name counter cmd...
    local name=$1 c=$2; shift 2
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/${name}_$c -o p -- "$@" > $O/${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; tail -5 $O/${name}_$c.log; return 1; }
    find $O/${name}_$c -name '*counter_collection.csv' > $O/${name}_$c.path
}
pipe_pass() {  # counter
    local c=$1 J=p$RANDOM$RANDOM
    RANK=1 WORLD_SIZE=2 LOCAL_RANK=1 LOCAL_WORLD_SIZE=2 MV2AMD_JOBID=$J MV2AMD_TIMEOUT_S=40 MV2AMD_DEVICE=0 timeout -k 5 80 python3 tools/pmc_pipe.py > $O/pipe_r1_$c.log 2>&1 &
    local p1=$!
    RANK=0 WORLD_SIZE=2 LOCAL_RANK=0 LOCAL_WORLD_SIZE=2 MV2AMD_JOBID=$J MV2AMD_TIMEOUT_S=40 MV2AMD_DEVICE=0 pmc pipe $c python3 tools/pmc_pipe.py
    local r0=$?
    wait $p1
    local r1=$?
    [ $r0 = 0 ] && [ $r1 = 0 ] || { echo "pipe pass $c failed ($r0 $r1)"; tail -5 $O/pipe_r1_$c.log; return 1; }
}
pipe_pass FETCH_SIZE || exit 1
pipe_pass WRITE_SIZE || exit 1
python tools/pmc_summary.py "$(cat $O/pipe_FETCH_SIZE.path)" "$(cat $O/pipe_WRITE_SIZE.path)" "k_pipe<mv2::R<2, 8" $O/pmc_pipe.json 268435456 6 && cat $O/pmc_pipe.json
