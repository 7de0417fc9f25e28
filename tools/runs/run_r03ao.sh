set -o pipefail
# Round 3, pass ao: OSU-style validated sweeps through libmpi.so above 8 ranks on emulated nodes
# (one shared GPU, nodes linked over 127.0.0.1): allreduce 8 B - 16 MiB at 12 ranks as 6x2 and
# 12x1, reduce_scatter at 12x1 (the message schedules of the flat algorithms)
O=gpurun_out/r03ao
mkdir -p $O
run() {  # name ranks nodes args...
  local name=$1 n=$2 k=$3; shift 3
  timeout -k 10 280 python -m mvapich2_amd.mv2run -n $n --nodes $k --share-gpu --timeout 270 ./tools/osu/osu_coll "$@" -v > $O/$name.txt 2>&1 || { echo "$name failed"; tail -20 $O/$name.txt; return 1; }
  echo "== $name"; grep -v "^#" $O/$name.txt | awk 'NR%3==1'
}
run ar12_6x2 12 6 -c allreduce -m 8:16777216 -i 50 && run ar12_12x1 12 12 -c allreduce -m 8:16777216 -i 50 && \
run rs12_12x1 12 12 -c reduce_scatter -m 8:16777216 -i 50
