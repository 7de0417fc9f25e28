set -o pipefail
# Round 3, pass s: 8-byte..8 KiB allreduce latency (OSU loop in C, 2 and 8 ranks on the shared GPU)
# against the lingering window (MV2AMD_LINGER_US = 0 / 20 / 100 / 500).
O=gpurun_out/r03s
mkdir -p $O
for W in 0 20 100 500; do
  MV2AMD_LINGER_US=$W timeout -k 10 120 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 110 ./tools/osu/osu_coll -c allreduce -m 8:8192 -i 2000 > $O/osu_ar2_w$W.txt 2>&1 || { tail -20 $O/osu_ar2_w$W.txt; exit 1; }
  echo "== 2 ranks, window $W us"; cat $O/osu_ar2_w$W.txt | grep -v "^#" | head -12
done
for W in 0 100; do
  MV2AMD_LINGER_US=$W timeout -k 10 180 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 170 ./tools/osu/osu_coll -c allreduce -m 8:1024 -i 1000 > $O/osu_ar8_w$W.txt 2>&1 || { tail -20 $O/osu_ar8_w$W.txt; exit 1; }
  echo "== 8 ranks, window $W us"; grep -v "^#" $O/osu_ar8_w$W.txt | head -10
done
for W in 0 100; do
  MV2AMD_LINGER_US=$W timeout -k 10 120 ./tools/osu/osu_coll -c reduce_local -m 8:8 -i 5000 > $O/osu_rl_w$W.txt 2>&1 || { tail -20 $O/osu_rl_w$W.txt; exit 1; }
  echo "== reduce_local, window $W"; grep -v "^#" $O/osu_rl_w$W.txt | head -3
done
