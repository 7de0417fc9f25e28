set -o pipefail
# Round 5, pass x: element-wise one-shot reduce-scatter for small blocks off 16-byte boundaries
# (self-test block of 12 bytes): OSU reduce_scatter 4 B .. 64 KiB at 2 / 4 shared ranks, then the
# collective tests
O=gpurun_out/r05x
mkdir -p $O
export TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 200 python -m mvapich2_amd.mv2run -n $n --share-gpu --timeout 190 tools/osu/osu_coll -c reduce_scatter -m 4:65536 -i 500 -x 50 -v > $O/osu_reduce_scatter_${n}.txt 2>&1 || { tail -20 $O/osu_reduce_scatter_${n}.txt; exit 1; }
  grep -v MPI_Init $O/osu_reduce_scatter_${n}.txt | head -20
done
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread \
  tests/test_gpu_collectives_mp.py tests/test_gpu_mpich_coll_suite.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
