set -o pipefail
# Round 4: the pipelined kernel's smallest per-workgroup tile (16 KiB default) vs 8 and 4 KiB at 512 KiB - 8 MiB
O=gpurun_out/r04ps
mkdir -p $O
export TMPDIR=/tmp
for nr in 2 4; do
  for ms in 16384 8192 4096; do
    MV2AMD_PIPE_MIN_SUB=$ms timeout -k 10 200 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 190 tools/osu/osu_coll -c allreduce -m 524288:8388608 -i 300 -x 30 -v > $O/osu_${nr}share_$ms.txt 2>&1 || { tail $O/osu_${nr}share_$ms.txt; exit 1; }
    echo "== $nr ranks, min sub $ms"; grep -E "^[0-9]" $O/osu_${nr}share_$ms.txt
  done
done
