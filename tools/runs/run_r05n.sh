set -o pipefail
# Round 5, pass n: where the one-shot allreduce stops paying on the shared GPU: OSU allreduce /
# allgather / bcast 64 KiB .. 4 MiB with the one-shot limit at 256 KiB (default) and 1 MiB
# (MV2AMD_ONESHOT_MAX), 2 and 4 shared ranks
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
for n in 2 4; do
  for lim in 262144 1048576 2097152; do
    MV2AMD_ONESHOT_MAX=$lim timeout -k 10 200 python -m mvapich2_amd.mv2run -n $n --share-gpu --timeout 190 tools/osu/osu_coll -c allreduce -m 65536:4194304 -i 200 -x 20 -v > $O/ar_${n}_${lim}.txt 2>&1 || { tail -20 $O/ar_${n}_${lim}.txt; exit 1; }
  done
  paste $O/ar_${n}_262144.txt $O/ar_${n}_1048576.txt $O/ar_${n}_2097152.txt | grep -v MPI_Init | awk '{print $1, $2, $7, $12, $5, $10, $15}'
done
