set -o pipefail
# Round 5, pass bb: the compact element-wise one-shot reduce-scatter kernel: 8-byte host profile at 2
# shared ranks (r05ay before: launch -> completion 9.05 us), OSU reduce_scatter 4 B - 8 KiB at 2 / 4
# ranks (the vector body for aligned operands from MV2AMD_RS_SCALAR_MAX=0 beside the default), then the
# collective tests
O=gpurun_out/r05bb
mkdir -p $O
export TMPDIR=/tmp
MV2AMD_HOST_PROFILE=500 timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c reduce_scatter -m 8:8 -i 5000 -x 500 > $O/rs_hp.txt 2>&1 || { tail -20 $O/rs_hp.txt; exit 1; }
grep -v "^#" $O/rs_hp.txt | head -4
for n in 2 4; do
  for sm in 0 4096; do
    MV2AMD_RS_SCALAR_MAX=$sm timeout -k 10 200 python -m mvapich2_amd.mv2run -n $n --share-gpu --timeout 190 tools/osu/osu_coll -c reduce_scatter -m 4:8192 -i 3000 -x 300 -v > $O/rs_${n}_${sm}.txt 2>&1 || { tail -20 $O/rs_${n}_${sm}.txt; exit 1; }
  done
  echo "== $n ranks: size, scalar_max 0 / 4096 (us)"
  paste $O/rs_${n}_0.txt $O/rs_${n}_4096.txt | grep -v "MPI_Init\|^#" | awk '{print $1, $2, $7, $5, $10}'
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_collectives_mp.py tests/test_gpu_multinode_mp.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
