set -o pipefail
# Round 4: one-shot grid at one 16-B vector per thread (256 per workgroup, up to 64 workgroups): the whole -m gpu suite, then the OSU allreduce sweeps at 2 and 4 shared ranks
O=gpurun_out/r04os
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for nr in 2 4; do
  timeout -k 10 280 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 270 tools/osu/osu_coll -c allreduce -m 8:1073741824 -i 200 -x 20 -v > $O/osu_allreduce_${nr}share.txt 2>&1 || { tail $O/osu_allreduce_${nr}share.txt; exit 1; }
done
head -n 24 $O/osu_allreduce_2share.txt | tail -n 21; head -n 24 $O/osu_allreduce_4share.txt | tail -n 21
