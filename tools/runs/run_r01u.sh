set -o pipefail
# Owner hoisted out of the butterfly reduce loops, user-op ring order: GPU tests, then the OSU allreduce / reduce
# size sweeps through libmpi.so (2 and 8 ranks sharing the one GPU) across the two-level / butterfly / ring regimes.
O=gpurun_out/r01u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 ./tools/osu/osu_coll -c allreduce -m 8:268435456 -i 50 -x 5 -v > $O/osu_allreduce_2.txt 2>&1 || { tail $O/osu_allreduce_2.txt; exit 1; }
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 190 ./tools/osu/osu_coll -c allreduce -m 8:67108864 -i 20 -x 3 -v > $O/osu_allreduce_8.txt 2>&1 || { tail $O/osu_allreduce_8.txt; exit 1; }
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 ./tools/osu/osu_coll -c reduce -m 1024:67108864 -i 20 -x 3 > $O/osu_reduce_2.txt 2>&1 || { tail $O/osu_reduce_2.txt; exit 1; }
cat $O/osu_allreduce_2.txt $O/osu_allreduce_8.txt $O/osu_reduce_2.txt
