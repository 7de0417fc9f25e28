set -o pipefail
# Round 4: OSU-loop sweeps through libmpi.so with the current build (configs[2]: allreduce 8 B - 1 GiB,
# validated; configs[3]: reduce_scatter / allgather / bcast to 256 MiB) at 2 and 4 ranks on one GPU
O=gpurun_out/r04osu
mkdir -p $O
export TMPDIR=/tmp
for nr in 2 4; do
  timeout -k 10 280 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 270 tools/osu/osu_coll -c allreduce -m 8:1073741824 -i 20 -x 5 -v > $O/osu_allreduce_${nr}share.txt 2>&1 || { tail $O/osu_allreduce_${nr}share.txt; exit 1; }
  for c in reduce_scatter allgather bcast; do
    timeout -k 10 200 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 190 tools/osu/osu_coll -c $c -m 8:268435456 -i 20 -x 5 -v > $O/osu_${c}_${nr}share.txt 2>&1 || { tail $O/osu_${c}_${nr}share.txt; exit 1; }
  done
done
tail -n 4 $O/osu_allreduce_2share.txt; tail -n 4 $O/osu_allreduce_4share.txt
