set -o pipefail
# host cost of hipLaunchKernelGGL: argument size, libmpi.so's code object, kernarg placement
O=gpurun_out/r02i
mkdir -p $O
timeout -k 5 60 ./tools/launch_probe2 > $O/plain.txt 2>&1 || { cat $O/plain.txt; exit 1; }
cat $O/plain.txt
timeout -k 5 60 ./tools/launch_probe2 mvapich2_amd/lib/libmpi.so > $O/with_libmpi.txt 2>&1 || { cat $O/with_libmpi.txt; exit 1; }
cat $O/with_libmpi.txt
HIP_FORCE_DEV_KERNARG=0 timeout -k 5 60 ./tools/launch_probe2 > $O/hostkernarg.txt 2>&1 || { cat $O/hostkernarg.txt; exit 1; }
cat $O/hostkernarg.txt
HIP_FORCE_DEV_KERNARG=1 timeout -k 5 60 ./tools/launch_probe2 > $O/devkernarg.txt 2>&1 || { cat $O/devkernarg.txt; exit 1; }
cat $O/devkernarg.txt
