set -o pipefail
O=gpurun_out/r03g
mkdir -p $O
for n in 2 3 4 8; do
  timeout -k 10 200 python -m mvapich2_amd.mv2run -n $n --share-gpu --timeout 180 ./tests/mpich_coll/coll_suite device red3 red4 longuser coll8 coll9 coll10 coll12 iallred nonblocking2 > $O/suite_dev$n.txt 2>&1 || { echo "n=$n failed"; tail -30 $O/suite_dev$n.txt; exit 1; }
  grep -v " 0 " $O/suite_dev$n.txt || true
done
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 3 --share-gpu --timeout 180 ./tests/mpich_coll/coll_suite host red3 red4 longuser coll8 coll9 coll10 coll12 iallred nonblocking2 > $O/suite_host3.txt 2>&1 || { echo "host failed"; tail -30 $O/suite_host3.txt; exit 1; }
cat $O/suite_dev4.txt $O/suite_host3.txt
