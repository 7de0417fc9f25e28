set -o pipefail
# Round 4: host-side split (entry -> launch, launch, launch -> done) of small reduce_scatter_block vs allreduce at 2 shared ranks
O=gpurun_out/r04lat6
mkdir -p $O
export TMPDIR=/tmp
for c in allreduce reduce_scatter_block bcast; do
  MV2AMD_HOST_PROFILE=400 LAT_COLL=$c LAT_SIZES=512 LAT_ITERS=2000 timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 python -u tools/lat_sizes.py > $O/lat_$c.txt 2>&1 || { tail -20 $O/lat_$c.txt; exit 1; }
  echo "== $c"; grep -E " B |host profile" $O/lat_$c.txt
done
