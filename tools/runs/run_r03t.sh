set -o pipefail
# Round 3, pass t: lingering one-shot diagnostics at 2 ranks (posts / launches counters; with and
# without the null-stream idle check) and the 1-rank Reduce_local floor.
O=gpurun_out/r03t
mkdir -p $O
export MV2AMD_LINGER_STATS=1 MV2AMD_HOST_PROFILE=1
for NC in 1 0; do
  MV2AMD_LINGER_NULLCHECK=$NC MV2AMD_LINGER_US=500 timeout -k 10 100 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 90 ./tools/osu/osu_coll -c allreduce -m 8:64 -i 2000 > $O/osu_ar2_nc$NC.txt 2>&1 || { tail -20 $O/osu_ar2_nc$NC.txt; exit 1; }
  echo "== 2 ranks window 500 nullcheck $NC"; cat $O/osu_ar2_nc$NC.txt | grep -v "^#"
done
