set -o pipefail
# Round 4, pass d: the 5-rank host-operand redscat3 / redscatblk3 cases that ran 39 s in r04a, alone
# and after the suite's preceding cases, with beacon histories printed on a device-wait timeout.
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
export MV2AMD_TIMEOUT_S=30 PYTHONPATH=$PWD
timeout -k 10 150 python3 -m mvapich2_amd.mv2run -n 5 --share-gpu --timeout 140 tests/mpich_coll/coll_suite host redscat3 redscatblk3 > $O/alone.out 2> $O/alone.err; echo "alone rc $?"
cat $O/alone.out
timeout -k 10 150 python3 -m mvapich2_amd.mv2run -n 5 --share-gpu --timeout 140 tests/mpich_coll/coll_suite host allred2 allred3 allred4 allred5 allred6 allredmany uoplong redscat2 red_scat_block2 redscat3 redscatblk3 > $O/prefix.out 2> $O/prefix.err; echo "prefix rc $?"
cat $O/prefix.out
grep -c "error" $O/alone.err $O/prefix.err || true
