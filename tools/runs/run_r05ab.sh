set -o pipefail
# Round 5, pass ab: diagnosis of the r05aa mismatch (test_random_sequence_across_nodes[12-4-9000],
# case rn9023: flat-ring allreduce PROD int32 700003 over 3 emulated nodes of 4, rank 0 one element):
# the ring path alone, 150 calls at 12 = 3 x 4 with point-to-point copy kernels, then copy engines
O=gpurun_out/r05ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u tools/ringsoak_diag.py 12 4 150 31 > $O/kcopy.json 2> $O/kcopy.err || { tail -30 $O/kcopy.err; exit 1; }
cat $O/kcopy.json
MV2AMD_P2P_KERNEL_COPY=0 timeout -k 10 420 python -u tools/ringsoak_diag.py 12 4 150 31 > $O/sdma.json 2> $O/sdma.err || { tail -30 $O/sdma.err; exit 1; }
cat $O/sdma.json
