set -o pipefail
# Round 3, pass ap: does the OSU harness run across emulated nodes?  4 ranks as 2x2, then 12 as
# 6x2, small sizes, line-buffered output so progress shows
O=gpurun_out/r03ap
mkdir -p $O
run() {  # name ranks nodes args...
  local name=$1 n=$2 k=$3; shift 3
  timeout -k 10 120 python -m mvapich2_amd.mv2run -n $n --nodes $k --share-gpu --timeout 110 stdbuf -oL -eL ./tools/osu/osu_coll "$@" -v > $O/$name.txt 2>&1 || { echo "$name failed"; tail -30 $O/$name.txt; return 1; }
  echo "== $name"; grep -v "^#" $O/$name.txt | head -40
}
run ar4_2x2 4 2 -c allreduce -m 8:65536 -i 20 && run ar12_6x2 12 6 -c allreduce -m 8:65536 -i 20
