set -o pipefail
# Round 4: one-shot at one vector per thread (up to 64 workgroups) and 4 KiB minimum pipe tiles: the whole -m gpu suite, OSU sweeps at 2 / 4 shared ranks, the N = 1 line and the 2-rank rehearsal
O=gpurun_out/r04pt
mkdir -p $O
export TMPDIR=/tmp
export MV2AMD_PIPE_MIN_SUB=4096  # the candidate default, under every step
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for nr in 2 4; do
  timeout -k 10 280 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 270 tools/osu/osu_coll -c allreduce -m 8:1073741824 -i 200 -x 20 -v > $O/osu_allreduce_${nr}share.txt 2>&1 || { tail $O/osu_allreduce_${nr}share.txt; exit 1; }
  for c in reduce_scatter allgather bcast; do
    timeout -k 10 200 python -m mvapich2_amd.mv2run -n $nr --share-gpu --timeout 190 tools/osu/osu_coll -c $c -m 8:268435456 -i 100 -x 10 -v > $O/osu_${c}_${nr}share.txt 2>&1 || { tail $O/osu_${c}_${nr}share.txt; exit 1; }
  done
done
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
cut -c1-200 $O/bench_n1.json $O/bench_torchrun2.json
grep -E "^(8|8192|65536|262144|524288|1048576|2097152|268435456|1073741824) " $O/osu_allreduce_2share.txt $O/osu_allreduce_4share.txt
