set -o pipefail
# HIP API time per call inside the library's small-message paths
O=gpurun_out/r02j
mkdir -p $O
export TMPDIR=/tmp MV2AMD_HOST_PROFILE=1
timeout -k 5 120 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/rl -o rl -- ./tools/osu/osu_coll -c reduce_local -m 8:8 -i 3000 > $O/rl.txt 2>&1 || { tail -20 $O/rl.txt; exit 1; }
cat $O/rl.txt
find $O/rl -name '*stats.csv'
