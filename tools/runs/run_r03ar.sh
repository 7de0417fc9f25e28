set -o pipefail
# Round 3, pass ar: the 12x1 OSU allreduce again with GPU_MAX_HW_QUEUES=2 per process (12 x 2
# hardware queues instead of 12 x 4: do the emulated nodes' processes stop being time-sliced?)
O=gpurun_out/r03ar
mkdir -p $O
export GPU_MAX_HW_QUEUES=2
timeout -k 10 150 python -m mvapich2_amd.mv2run -n 12 --nodes 12 --share-gpu --timeout 140 stdbuf -oL -eL ./tools/osu/osu_coll -c allreduce -m 8:4194304 -i 20 -v > $O/ar12_12x1_q2.txt 2>&1 || { echo "failed"; tail -30 $O/ar12_12x1_q2.txt; exit 1; }
grep -v "^#" $O/ar12_12x1_q2.txt
