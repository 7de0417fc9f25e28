set -o pipefail
# Round 4: OSU allreduce and reduce_scatter to 4 MiB at 8 ranks sharing one GPU, final build
O=gpurun_out/r04o8
mkdir -p $O
export TMPDIR=/tmp
for c in allreduce reduce_scatter; do
  timeout -k 10 280 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 270 tools/osu/osu_coll -c $c -m 8:4194304 -i 200 -x 20 -v > $O/osu_${c}_8share.txt 2>&1 || { tail $O/osu_${c}_8share.txt; exit 1; }
  echo "== $c"; grep -E "^[0-9]" $O/osu_${c}_8share.txt
done
