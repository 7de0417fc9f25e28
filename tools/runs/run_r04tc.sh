set -o pipefail
# Round 4: a call's last device-to-device copy as a kernel that raises the completion word (was hipMemcpyAsync + stream synchronisation): OSU reduce_scatter / bcast / allreduce at 2 and 4 shared ranks, then the whole -m gpu suite
O=gpurun_out/r04tc
mkdir -p $O
export TMPDIR=/tmp
for nr in 2 4; do
  for c in reduce_scatter bcast allreduce; do
    timeout -k 10 200 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 190 tools/osu/osu_coll -c $c -m 8:8388608 -i 300 -x 30 -v > $O/osu_${c}_${nr}share.txt 2>&1 || { tail $O/osu_${c}_${nr}share.txt; exit 1; }
  done
done
grep -E "^(8|64|512|4096|65536|1048576) " $O/osu_reduce_scatter_2share.txt $O/osu_reduce_scatter_4share.txt $O/osu_bcast_2share.txt
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
