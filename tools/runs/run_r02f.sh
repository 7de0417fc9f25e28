set -o pipefail
# 8-byte allreduce latency: plain 2-rank probe, then both ranks under
# rocprofv3 --kernel-trace for the kernel / skew / host-gap breakdown.
O=gpurun_out/r02f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 110 python -u tools/lat_probe.py > $O/lat_plain.txt 2>&1 || { tail -20 $O/lat_plain.txt; exit 1; }
cat $O/lat_plain.txt
J=l$RANDOM$RANDOM
for r in 0 1; do
    RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r LOCAL_WORLD_SIZE=2 MV2AMD_JOBID=$J MV2AMD_TIMEOUT_S=40 timeout -k 5 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr$r -o lat -- python3 tools/lat_probe.py > $O/lat_tr$r.txt 2>&1 &
done
wait %1; r0=$?
wait %2; r1=$?
[ $r0 = 0 ] && [ $r1 = 0 ] || { echo "traced run failed $r0 $r1"; tail -5 $O/lat_tr0.txt $O/lat_tr1.txt; exit 1; }
grep rank $O/lat_tr0.txt $O/lat_tr1.txt
python tools/lat_breakdown.py $O/lat_breakdown.json $(find $O/tr0 -name '*kernel_trace.csv') $(find $O/tr1 -name '*kernel_trace.csv')
