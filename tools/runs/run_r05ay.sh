set -o pipefail
# Round 5, pass ay: where the 8-byte reduce_scatter's extra 1.5 us over allreduce goes (host
# profile: entry -> launch, launch, launch -> completion word), 2 shared ranks
O=gpurun_out/r05ay
mkdir -p $O
export TMPDIR=/tmp
for c in allreduce reduce_scatter allgather bcast; do
  MV2AMD_HOST_PROFILE=500 timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c $c -m 8:8 -i 5000 -x 500 > $O/$c.txt 2>&1 || { tail -20 $O/$c.txt; exit 1; }
  echo "== $c"; grep -v "^#" $O/$c.txt | grep -i -E "^ *8 |profile|entry|launch" | head -8
done
