set -o pipefail
# Round 4, pass e: the prefix sequence of r04d with MV2AMD_DEBUG=1 (every pipelined launch's mode,
# grid, tsub, rounds and maxlen per rank, plus the plans), to compare the ranks' launches call by call.
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
export MV2AMD_TIMEOUT_S=30 PYTHONPATH=$PWD MV2AMD_DEBUG=1
timeout -k 10 150 python3 -m mvapich2_amd.mv2run -n 5 --share-gpu --timeout 140 tests/mpich_coll/coll_suite host allred2 allred3 allred4 allred5 allred6 allredmany uoplong redscat2 red_scat_block2 redscat3 redscatblk3 > $O/prefix.out 2> $O/prefix.err; echo "prefix rc $?"
cat $O/prefix.out
wc -l $O/prefix.err
gzip -f $O/prefix.err
