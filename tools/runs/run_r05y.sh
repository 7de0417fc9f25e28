set -o pipefail
# Round 5, pass y: one-shot reduce-scatter, vector body vs element-wise body for small aligned
# operands (MV2AMD_RS_SCALAR_MAX), OSU reduce_scatter 4 B .. 16 KiB at 2 / 4 shared ranks
O=gpurun_out/r05y
mkdir -p $O
export TMPDIR=/tmp
for n in 2 4; do
  for sm in 0 4096; do
    MV2AMD_RS_SCALAR_MAX=$sm timeout -k 10 200 python -m mvapich2_amd.mv2run -n $n --share-gpu --timeout 190 tools/osu/osu_coll -c reduce_scatter -m 4:16384 -i 1000 -x 100 -v > $O/rs_${n}_${sm}.txt 2>&1 || { tail -20 $O/rs_${n}_${sm}.txt; exit 1; }
  done
  paste $O/rs_${n}_0.txt $O/rs_${n}_4096.txt | grep -v MPI_Init | awk '{print $1, $2, $7, $5, $10}'
done
