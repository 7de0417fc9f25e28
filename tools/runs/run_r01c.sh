set -o pipefail
mkdir -p gpurun_out/r01c
timeout -k 10 120 tools/uc_bw > gpurun_out/r01c/uc_bw.txt 2>&1 && \
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 220 tools/osu/osu_coll -c allreduce -m 8:268435456 -i 20 -x 5 -v > gpurun_out/r01c/osu_ar_2share.txt 2>&1 && \
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 4 --share-gpu --timeout 220 tools/osu/osu_coll -c allreduce -m 8:268435456 -i 20 -x 5 -v > gpurun_out/r01c/osu_ar_4share.txt 2>&1
cat gpurun_out/r01c/uc_bw.txt gpurun_out/r01c/osu_ar_2share.txt gpurun_out/r01c/osu_ar_4share.txt
