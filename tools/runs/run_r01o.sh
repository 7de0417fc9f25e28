set -o pipefail
# smoke(), p2p tests at 2/3/8 ranks, OSU pt2pt latency/bw through the C harness (2 ranks, one GPU)
O=gpurun_out/r01o
mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_p2p_mp.py -x -v --timeout 200 --timeout-method thread > $O/p2p.log 2>&1 || { tail -30 $O/p2p.log; exit 1; }
tail -2 $O/p2p.log
timeout -k 10 120 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 110 ./tools/osu/osu_coll -c latency -m 8:4194304 -i 200 -x 20 > $O/osu_latency.txt 2>&1 || { tail $O/osu_latency.txt; exit 1; }
timeout -k 10 120 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 110 ./tools/osu/osu_coll -c bw -m 4096:16777216 -i 10 -x 2 > $O/osu_bw.txt 2>&1 || { tail $O/osu_bw.txt; exit 1; }
cat $O/osu_latency.txt $O/osu_bw.txt
