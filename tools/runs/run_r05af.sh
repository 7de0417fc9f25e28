set -o pipefail
# Round 5, pass af: L2 staleness probe (tools/diag/l2_probe): a copy on stream B, the host
# synchronises B, a kernel on stream A reads the buffer its XCDs had cached; alone, then with
# 8 processes at once
O=gpurun_out/r05af
mkdir -p $O
for m in 0 1 2 3; do timeout -k 10 120 tools/diag/l2_probe $m 300 > $O/alone_$m.json 2>&1 || { cat $O/alone_$m.json; exit 1; }; cat $O/alone_$m.json; done
for m in 0 2; do
  pids=""
  for i in $(seq 1 8); do timeout -k 10 240 tools/diag/l2_probe $m 300 > $O/loaded_${m}_$i.json 2>&1 & pids="$pids $!"; done
  rc=0; for p in $pids; do wait $p || rc=1; done
  cat $O/loaded_${m}_*.json
  [ $rc = 0 ] || exit 1
done
