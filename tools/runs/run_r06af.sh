#!/bin/bash
set -o pipefail
# Round 6, pass af: A/B of the compact one-shot kernels run as one wave up to 64 elements (no workgroup barrier before the completion word)
# -- OSU 8 B .. 2 KiB at 2 ranks sharing the GPU; A = the library before (abtest/, by
# LD_LIBRARY_PATH over osu_coll's RUNPATH), B = in-tree
O=gpurun_out/r06af
mkdir -p $O
for k in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export LD_LIBRARY_PATH=$PWD/abtest; else unset LD_LIBRARY_PATH; fi
    timeout -k 10 150 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 140 tools/osu/osu_coll -c all -m 8:2048 -f 4 -i 2000 -x 200 -v > $O/osu_${v}$k.txt 2>&1 || { tail -20 $O/osu_${v}$k.txt; exit 1; }
    echo "== $v$k"; grep -v "^JSON\|^#" $O/osu_${v}$k.txt | head -40
  done
done
