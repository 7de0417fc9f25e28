set -o pipefail
# Round 4: one-shot kernel with batched loads; one vector per thread (256 per workgroup, default) vs 512 per workgroup
O=gpurun_out/r04lat3
mkdir -p $O
export TMPDIR=/tmp
for nr in 2 4; do
  for vpw in 256 512; do
    MV2AMD_ONESHOT_VECS_PER_WG=$vpw timeout -k 10 240 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 230 python -u tools/lat_sizes.py > $O/lat_${nr}share_$vpw.txt 2>&1 || { tail -20 $O/lat_${nr}share_$vpw.txt; exit 1; }
    echo "== $nr ranks, $vpw vectors per workgroup"; grep " B " $O/lat_${nr}share_$vpw.txt
  done
done
