set -o pipefail
# Round 5, pass ae: the r05ab diagnosis again with spans (r05ad's box showed no mismatch in 150 calls):
# 300 calls with copy kernels, 300 with copy engines
O=gpurun_out/r05ae
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u tools/ringsoak_diag.py 12 4 300 31 > $O/kcopy.json 2> $O/kcopy.err || { tail -30 $O/kcopy.err; exit 1; }
cat $O/kcopy.json
MV2AMD_P2P_KERNEL_COPY=0 timeout -k 10 420 python -u tools/ringsoak_diag.py 12 4 300 32 > $O/sdma.json 2> $O/sdma.err || { tail -30 $O/sdma.err; exit 1; }
cat $O/sdma.json
