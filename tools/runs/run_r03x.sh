set -o pipefail
# Round 3, pass x: OSU-style sweeps through libmpi.so on the shared GPU (validated, -v):
# allreduce 8 B - 1 GiB at 2 ranks, 8 B - 256 MiB at 4 and 8 ranks; reduce_scatter / allgather /
# bcast 8 B - 256 MiB at 2 ranks.
O=gpurun_out/r03x
mkdir -p $O
run() {  # name ranks args...
  local name=$1 n=$2; shift 2
  timeout -k 10 280 python -m mvapich2_amd.mv2run -n $n --share-gpu --timeout 270 ./tools/osu/osu_coll "$@" -v > $O/$name.txt 2>&1 || { echo "$name failed"; tail -20 $O/$name.txt; return 1; }
  echo "== $name"; grep -v "^#" $O/$name.txt | awk 'NR%3==1'
}
run ar2 2 -c allreduce -m 8:1073741824 && run ar4 4 -c allreduce -m 8:268435456 && run ar8 8 -c allreduce -m 8:268435456 -i 300 && \
run rs2 2 -c reduce_scatter -m 8:268435456 && run ag2 2 -c allgather -m 8:268435456 && run bc2 2 -c bcast -m 8:268435456
