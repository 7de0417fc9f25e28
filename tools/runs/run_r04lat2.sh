set -o pipefail
# Round 4: small-message allreduce latency per size at 2 and 4 shared ranks: algorithm, wall, kernel time
O=gpurun_out/r04lat2
mkdir -p $O
export TMPDIR=/tmp
for nr in 2 4; do
  timeout -k 10 240 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 230 python -u tools/lat_sizes.py > $O/lat_${nr}share.txt 2>&1 || { tail -20 $O/lat_${nr}share.txt; exit 1; }
  grep " B " $O/lat_${nr}share.txt
done
