set -o pipefail
O=gpurun_out/r02l
mkdir -p $O
timeout -k 5 60 ./tools/launch_probe2 mvapich2_amd/lib/libmpi.so > $O/with_libmpi.txt 2>&1 || { cat $O/with_libmpi.txt; exit 1; }
cat $O/with_libmpi.txt
