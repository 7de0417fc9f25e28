set -o pipefail
# Round 4: reduce_scatter_block / bcast / allreduce small-message latency at 2 shared ranks: wall vs kernel time
O=gpurun_out/r04lat5
mkdir -p $O
export TMPDIR=/tmp
for c in allreduce reduce_scatter_block bcast; do
  LAT_COLL=$c LAT_SIZES=8,512,4096,65536 LAT_ITERS=1500 timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 python -u tools/lat_sizes.py > $O/lat_$c.txt 2>&1 || { tail -20 $O/lat_$c.txt; exit 1; }
  echo "== $c"; grep " B " $O/lat_$c.txt
done
