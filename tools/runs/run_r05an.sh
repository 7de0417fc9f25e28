set -o pipefail
# Round 5, pass an: cross-process visibility probe (tools/diag/ipc_probe.hip): a kernel in one
# process copies 4 MiB into another process's uncached IPC buffer, completes by word (mode 0),
# stream synchronisation (1) or system fence per workgroup + word (2); the owner checks every word.
# One pair alone, then 4 pairs at once
O=gpurun_out/r05an
mkdir -p $O
for m in 0 1 2; do
  timeout -k 10 120 tools/diag/ipc_probe r $m 1500 /mv2diag_$m > $O/alone_$m.json 2>&1 &
  rp=$!
  sleep 1
  timeout -k 10 120 tools/diag/ipc_probe w $m 1500 /mv2diag_$m || { echo "writer failed"; exit 1; }
  wait $rp || { cat $O/alone_$m.json; exit 1; }
  cat $O/alone_$m.json
done
for m in 0 1; do
  pids=""
  for i in 1 2 3 4; do
    timeout -k 10 200 tools/diag/ipc_probe r $m 1500 /mv2diagL_${m}_$i > $O/loaded_${m}_$i.json 2>&1 & pids="$pids $!"
  done
  sleep 1
  for i in 1 2 3 4; do timeout -k 10 200 tools/diag/ipc_probe w $m 1500 /mv2diagL_${m}_$i & pids="$pids $!"; done
  rc=0; for p in $pids; do wait $p || rc=1; done
  cat $O/loaded_${m}_*.json
  [ $rc = 0 ] || exit 1
done
