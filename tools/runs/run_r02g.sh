set -o pipefail
# light acquire + one-workgroup completion + NM-column pipe: full check, latency
# probe at 2 and 8 ranks, 2-rank shared-GPU bench line.
O=gpurun_out/r02g
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_check.sh r02g || exit 1
timeout -k 10 120 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 110 python -u tools/lat_probe.py > $O/lat2.txt 2>&1 || { tail -20 $O/lat2.txt; exit 1; }
cat $O/lat2.txt
LAT_ITERS=500 timeout -k 10 180 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 170 python -u tools/lat_probe.py > $O/lat8.txt 2>&1 || { tail -20 $O/lat8.txt; exit 1; }
cat $O/lat8.txt
timeout -k 10 240 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 230 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 300 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
