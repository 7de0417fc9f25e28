set -o pipefail
# Round 3, pass c: unpack write-side floors (pack_variants), pack/unpack call overhead on random
# data with kernel-trace stats, the whole -m gpu suite, N=1 bench with its kernel stats, 2-rank bench.
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/pack_variants > $O/pack_variants.txt 2> $O/pack_variants.err || { tail -5 $O/pack_variants.err; exit 1; }
cat $O/pack_variants.txt
timeout -k 10 120 ./tools/osu/pack_overhead > $O/pack_overhead.json 2> $O/pack_overhead.err || { tail -5 $O/pack_overhead.err; exit 1; }
cat $O/pack_overhead.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pack -o pack -- ./tools/osu/pack_overhead > $O/prof_pack.json 2> $O/prof_pack.err || { tail -20 $O/prof_pack.err; exit 1; }
find $O/prof_pack -name '*kernel_stats.csv' -exec cat {} \;
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -80 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
cat $O/bench_n1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec head -12 {} \;
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 290 python -u bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_2share.json 2> $O/bench_2share.err || { tail -20 $O/bench_2share.err; exit 1; }
cat $O/bench_2share.json
