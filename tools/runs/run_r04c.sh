set -o pipefail
# Round 4, pass c: the N = 1 bench under rocprofv3 --kernel-trace --stats (the kernel average of
# k_reduce_local for the line's roofline, and the bench's own MPI_Pack / MPI_Unpack loop launch by
# launch: VERDICT r03 item 5), then the plain N = 1 bench line.
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
cat $O/bench_n1.json | cut -c1-600
