set -o pipefail
# completion wait without stream queries + op table: full check, small-message host profile
O=gpurun_out/r02k
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_check.sh r02k || exit 1
export MV2AMD_HOST_PROFILE=1
timeout -k 10 120 ./tools/osu/osu_coll -c reduce_local -m 8:8 -i 5000 > $O/osu_rl8.txt 2>&1 || { tail -20 $O/osu_rl8.txt; exit 1; }
cat $O/osu_rl8.txt
timeout -k 10 120 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 110 ./tools/osu/osu_coll -c allreduce -m 8:1048576 > $O/osu_ar_2.txt 2>&1 || { tail -20 $O/osu_ar_2.txt; exit 1; }
cat $O/osu_ar_2.txt
timeout -k 10 180 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 170 ./tools/osu/osu_coll -c allreduce -m 8:65536 -i 500 > $O/osu_ar_8.txt 2>&1 || { tail -20 $O/osu_ar_8.txt; exit 1; }
cat $O/osu_ar_8.txt
