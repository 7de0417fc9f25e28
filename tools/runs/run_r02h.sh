set -o pipefail
# small-message host/device breakdown: host profile of the OSU allreduce loop
# (2 ranks) and of Reduce_local (1 rank).
O=gpurun_out/r02h
mkdir -p $O
export TMPDIR=/tmp MV2AMD_HOST_PROFILE=1
timeout -k 10 120 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 110 ./tools/osu/osu_coll -c allreduce -m 8:8 -i 5000 > $O/osu_ar8_2.txt 2>&1 || { tail -20 $O/osu_ar8_2.txt; exit 1; }
cat $O/osu_ar8_2.txt
timeout -k 10 120 ./tools/osu/osu_coll -c reduce_local -m 8:8 -i 5000 > $O/osu_rl8.txt 2>&1 || { tail -20 $O/osu_rl8.txt; exit 1; }
cat $O/osu_rl8.txt
timeout -k 10 120 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 110 ./tools/osu/osu_coll -c allreduce -m 8:1048576 > $O/osu_ar_2.txt 2>&1 || { tail -20 $O/osu_ar_2.txt; exit 1; }
cat $O/osu_ar_2.txt
