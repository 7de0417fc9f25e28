set -o pipefail
# Round 4, pass f: is the r04d/e stall (one rank's redscat3 kernel not dispatched for 30 s after the
# user-op case) hardware-queue oversubscription?  (A) the r04e prefix without uoplong (the only case
# that now creates each rank's point-to-point stream); (B) the full prefix with 2 HW queues per process.
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
export MV2AMD_TIMEOUT_S=30 PYTHONPATH=$PWD
S="python3 -m mvapich2_amd.mv2run -n 5 --share-gpu --timeout 140 tests/mpich_coll/coll_suite host"
timeout -k 10 150 $S allred2 allred3 allred4 allred5 allred6 allredmany redscat2 red_scat_block2 redscat3 redscatblk3 > $O/A.out 2> $O/A.err; echo "A rc $?"
cat $O/A.out
GPU_MAX_HW_QUEUES=2 timeout -k 10 150 $S allred2 allred3 allred4 allred5 allred6 allredmany uoplong redscat2 red_scat_block2 redscat3 redscatblk3 > $O/B.out 2> $O/B.err; echo "B rc $?"
cat $O/B.out
