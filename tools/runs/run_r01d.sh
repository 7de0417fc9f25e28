set -o pipefail
O=gpurun_out/r01d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for c in allreduce reduce_scatter allgather bcast reduce; do
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c $c -m 8:268435456 -i 20 -x 5 -v > $O/osu_${c}_2share.txt 2>&1 || { cat $O/osu_${c}_2share.txt | tail; exit 1; }
done
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 4 --share-gpu --timeout 190 tools/osu/osu_coll -c allreduce -m 8:268435456 -i 20 -x 5 -v > $O/osu_allreduce_4share.txt 2>&1
tail -n 12 $O/osu_*.txt
