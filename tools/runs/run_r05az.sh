set -o pipefail
# Round 5, pass az: the compact element-wise one-shot kernel (operands with no whole 16-byte
# vector): 8-byte allreduce host profile at 2 shared ranks, OSU allreduce / reduce 4-64 B at 2 and
# 4 ranks, then the collective parity tests
O=gpurun_out/r05az
mkdir -p $O
export TMPDIR=/tmp
MV2AMD_HOST_PROFILE=500 timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c allreduce -m 8:8 -i 5000 -x 500 > $O/allreduce_hp.txt 2>&1 || { tail -20 $O/allreduce_hp.txt; exit 1; }
grep -v "^#" $O/allreduce_hp.txt | head -4
for n in 2 4; do
  timeout -k 10 200 python -m mvapich2_amd.mv2run -n $n --share-gpu --timeout 190 tools/osu/osu_coll -c allreduce -m 4:64 -i 3000 -x 300 -v > $O/ar_$n.txt 2>&1 || { tail -20 $O/ar_$n.txt; exit 1; }
  echo "== $n ranks"; grep -v "^#\|MPI_Init" $O/ar_$n.txt | head -6
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_collectives_mp.py tests/test_gpu_reduce_local.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
