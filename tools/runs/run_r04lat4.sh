set -o pipefail
# Round 4: one-shot grid at one vector per thread: cap of 64 workgroups (default) vs 32
O=gpurun_out/r04lat4
mkdir -p $O
export TMPDIR=/tmp
for nr in 2 4; do
  for cap in 64 32; do
    MV2AMD_ONESHOT_MAX_WG=$cap timeout -k 10 240 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 230 python -u tools/lat_sizes.py > $O/lat_${nr}share_cap$cap.txt 2>&1 || { tail -20 $O/lat_${nr}share_cap$cap.txt; exit 1; }
    echo "== $nr ranks, cap $cap"; grep " B " $O/lat_${nr}share_cap$cap.txt
  done
done
