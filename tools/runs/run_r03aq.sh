set -o pipefail
# Round 3, pass aq: the OSU allreduce at 12 ranks as 12x1 (one rank per emulated node: no node-step
# kernels waiting on one another) against r03ap's 6x2
O=gpurun_out/r03aq
mkdir -p $O
timeout -k 10 150 python -m mvapich2_amd.mv2run -n 12 --nodes 12 --share-gpu --timeout 140 stdbuf -oL -eL ./tools/osu/osu_coll -c allreduce -m 8:4194304 -i 20 -v > $O/ar12_12x1.txt 2>&1 || { echo "failed"; tail -30 $O/ar12_12x1.txt; exit 1; }
grep -v "^#" $O/ar12_12x1.txt
