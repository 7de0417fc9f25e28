set -o pipefail
# Round 4: PMC HBM traffic of k_reduce_local (the bench's N = 1 kernel) for the current binary
# (block_done changed in r04y): FETCH_SIZE and WRITE_SIZE in separate passes, each under its own kill
O=gpurun_out/r04pmc
mkdir -p $O
export TMPDIR=/tmp
pmc() {  # name counter cmd...
    local name=$1 c=$2; shift 2
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/${name}_$c -o p -- "$@" > $O/${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; tail -5 $O/${name}_$c.log; return 1; }
    find $O/${name}_$c -name '*counter_collection.csv' > $O/${name}_$c.path
}
for c in FETCH_SIZE WRITE_SIZE; do pmc rl $c python3 tools/pmc_reduce_local.py || exit 1; done
python tools/pmc_summary.py "$(cat $O/rl_FETCH_SIZE.path)" "$(cat $O/rl_WRITE_SIZE.path)" "k_reduce_local<mv2::R<2, 8, void>, 2>" $O/pmc_reduce_local_r04pmc.json 805306368 6 && cat $O/pmc_reduce_local_r04pmc.json
