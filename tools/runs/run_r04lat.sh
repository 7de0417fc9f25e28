set -o pipefail
# Round 4: where the 2-rank allreduce latency steps up between 2 KiB and 8 KiB (host profile per size)
O=gpurun_out/r04lat
mkdir -p $O
export TMPDIR=/tmp
for s in 2048 4096 8192 16384 65536; do
  MV2AMD_HOST_PROFILE=1 timeout -k 10 120 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 110 tools/osu/osu_coll -c allreduce -m $s:$s -i 2000 -x 200 -v > $O/lat_$s.txt 2>&1 || { tail $O/lat_$s.txt; exit 1; }
done
for s in 2048 4096 8192 16384 65536; do grep -E "^[0-9]|host profile" $O/lat_$s.txt; done
