set -o pipefail
# Round 5, pass ad: the r05ab diagnosis with the wrong elements' spans (call, op, count, n wrong,
# first, last) for the first wrong calls, copy kernels only
O=gpurun_out/r05ad
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u tools/ringsoak_diag.py 12 4 150 31 > $O/kcopy.json 2> $O/kcopy.err || { tail -30 $O/kcopy.err; exit 1; }
cat $O/kcopy.json
