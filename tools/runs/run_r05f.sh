set -o pipefail
# Round 5, pass f: device point-to-point per-message cost: SDMA copy engines (default) against
# blit kernels (HSA_ENABLE_SDMA=0) for the chunk copies (osu_latency / osu_bw, 2 shared ranks)
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
for v in 1 0; do
  HSA_ENABLE_SDMA=$v timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c latency -m 8:16777216 -i 200 -I 20 > $O/lat_sdma$v.txt 2>&1 || { tail -20 $O/lat_sdma$v.txt; exit 1; }
  HSA_ENABLE_SDMA=$v timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c bw -m 8:16777216 -i 100 -I 10 > $O/bw_sdma$v.txt 2>&1 || { tail -20 $O/bw_sdma$v.txt; exit 1; }
done
paste $O/lat_sdma1.txt $O/lat_sdma0.txt
paste $O/bw_sdma1.txt $O/bw_sdma0.txt
