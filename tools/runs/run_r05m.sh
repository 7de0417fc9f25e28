set -o pipefail
# Round 5, pass m: one-shot allgather / broadcast for small messages: OSU sweeps at 2 and 4 shared
# ranks (8 B .. 4 MiB, validated), then the whole suite (self-test now 43 calls)
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
for n in 2 4; do
  for c in allgather bcast; do
    timeout -k 10 200 python -m mvapich2_amd.mv2run -n $n --share-gpu --timeout 190 tools/osu/osu_coll -c $c -m 8:4194304 -i 200 -x 20 -v > $O/osu_${c}_${n}.txt 2>&1 || { tail -20 $O/osu_${c}_${n}.txt; exit 1; }
  done
done
for n in 2 4; do paste $O/osu_allgather_$n.txt $O/osu_bcast_$n.txt | grep -v MPI_Init | cut -c1-150; done
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
