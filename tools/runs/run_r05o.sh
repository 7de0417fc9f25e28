set -o pipefail
# Round 5, pass o: the one-shot / pipelined probe up to the 1 MiB slot (forced on the shared GPU):
# the autotune test, then an OSU allreduce sweep with the autotune forced
O=gpurun_out/r05o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread tests/test_gpu_collectives_mp.py -k "autotune or hw_queue" > $O/pytest_autotune.log 2>&1 || { tail -60 $O/pytest_autotune.log; exit 1; }
tail -3 $O/pytest_autotune.log
MV2AMD_PIPE_AUTOTUNE=1 MV2AMD_PIPE_AUTOTUNE_BYTES=16777216 MV2AMD_INIT_REPORT=1 timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c allreduce -m 8192:4194304 -i 200 -x 20 -v > $O/ar_2_tuned.txt 2>&1 || { tail -20 $O/ar_2_tuned.txt; exit 1; }
cat $O/ar_2_tuned.txt
