set -o pipefail
# Round 5, pass g: point-to-point chunk copies as kernels with a completion word (default) against
# hipMemcpyAsync + stream synchronisation (MV2AMD_P2P_KERNEL_COPY=0): osu_latency / osu_bw at 2
# shared ranks; then the point-to-point GPU tests
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
for v in 0 1; do
  MV2AMD_P2P_KERNEL_COPY=$v timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c latency -m 8:16777216 -i 200 -I 20 > $O/lat_k$v.txt 2>&1 || { tail -20 $O/lat_k$v.txt; exit 1; }
  MV2AMD_P2P_KERNEL_COPY=$v timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c bw -m 8:16777216 -i 100 -I 10 > $O/bw_k$v.txt 2>&1 || { tail -20 $O/bw_k$v.txt; exit 1; }
done
paste $O/lat_k0.txt $O/lat_k1.txt | grep -v MPI_Init
paste $O/bw_k0.txt $O/bw_k1.txt | grep -v MPI_Init
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests/test_gpu_p2p_mp.py > $O/pytest_p2p.log 2>&1 || { echo "p2p tests failed"; tail -80 $O/pytest_p2p.log; exit 1; }
tail -2 $O/pytest_p2p.log
