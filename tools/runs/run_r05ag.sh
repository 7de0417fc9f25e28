set -o pipefail
# Round 5, pass ag: L2 staleness probe, host -> device copies (copy engines) followed by a kernel on
# another stream (modes 4-8 of tools/diag/l2_probe.hip), alone and with 8 processes at once
O=gpurun_out/r05ag
mkdir -p $O
for m in 4 5 6 7 8; do timeout -k 10 120 tools/diag/l2_probe $m 300 > $O/alone_$m.json 2>&1 || { cat $O/alone_$m.json; exit 1; }; cat $O/alone_$m.json; done
for m in 4 6; do
  pids=""
  for i in $(seq 1 8); do timeout -k 10 240 tools/diag/l2_probe $m 300 > $O/loaded_${m}_$i.json 2>&1 & pids="$pids $!"; done
  rc=0; for p in $pids; do wait $p || rc=1; done
  cat $O/loaded_${m}_*.json
  [ $rc = 0 ] || exit 1
done
