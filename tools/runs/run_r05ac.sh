set -o pipefail
# Round 5, pass ac: XCD placement probe (tools/diag/xcd_probe): do blocks with equal b % 8 share an
# XCD, alone and with 12 processes launching at once?
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 120 tools/diag/xcd_probe 2000 > $O/alone.json 2>&1 || { cat $O/alone.json; exit 1; }
cat $O/alone.json
pids=""
for i in $(seq 1 12); do timeout -k 10 240 tools/diag/xcd_probe 2000 > $O/loaded_$i.json 2>&1 & pids="$pids $!"; done
rc=0; for p in $pids; do wait $p || rc=1; done
cat $O/loaded_*.json
exit $rc
