set -o pipefail
# Round 3, pass am: PMC HBM traffic of the round-end tree's hot kernels (separate FETCH_SIZE /
# WRITE_SIZE passes, tools/pmc_summary.py corrections): Reduce_local (the N=1 value's kernel),
# pack and unpack on the configs[4] vector
O=gpurun_out/r03am
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
