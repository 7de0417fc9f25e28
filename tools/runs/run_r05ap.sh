set -o pipefail
# Round 5, pass ap: pageable host -> device hipMemcpy, then a kernel and a device -> host copy of
# the same bytes (tools/diag/upload_probe.hip): alone, then 12 processes at once (the soak's load)
O=gpurun_out/r05ap
mkdir -p $O
timeout -k 10 120 tools/diag/upload_probe 500 > $O/alone.json 2>&1 || { cat $O/alone.json; exit 1; }
cat $O/alone.json
pids=""
for i in $(seq 1 12); do timeout -k 10 240 tools/diag/upload_probe 400 > $O/loaded_$i.json 2>&1 & pids="$pids $!"; done
rc=0; for p in $pids; do wait $p || rc=1; done
cat $O/loaded_*.json
exit $rc
