set -o pipefail
# Round 4: one-shot reduce-scatter for small messages (each peer pushed only its block, one flag exchange): reduce-scatter GPU tests, OSU reduce_scatter at 2 / 4 shared ranks, then the whole -m gpu suite
O=gpurun_out/r04rs
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests -k "reduce_scatter or redscat or rs_" > $O/pytest_rs.log 2>&1 || { echo "rs tests failed"; tail -80 $O/pytest_rs.log; exit 1; }
tail -n 2 $O/pytest_rs.log
for nr in 2 4; do
  timeout -k 10 200 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 190 tools/osu/osu_coll -c reduce_scatter -m 8:8388608 -i 300 -x 30 -v > $O/osu_reduce_scatter_${nr}share.txt 2>&1 || { tail $O/osu_reduce_scatter_${nr}share.txt; exit 1; }
  LAT_COLL=reduce_scatter_block LAT_SIZES=8,512,4096,65536,262144 LAT_ITERS=1500 timeout -k 10 200 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 190 python -u tools/lat_sizes.py > $O/lat_rsb_${nr}share.txt 2>&1 || { tail -20 $O/lat_rsb_${nr}share.txt; exit 1; }
done
grep -E "^[0-9]" $O/osu_reduce_scatter_2share.txt $O/osu_reduce_scatter_4share.txt | head -40
grep " B " $O/lat_rsb_2share.txt $O/lat_rsb_4share.txt
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
