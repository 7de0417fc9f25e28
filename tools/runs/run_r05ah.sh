set -o pipefail
# Round 5, pass ah: the multi-node ring mismatch (r05ab / r05ae), A/B on one box: operands uploaded
# with hipMemcpy (pageable) as before, and with a device synchronisation after each upload
O=gpurun_out/r05ah
mkdir -p $O
export TMPDIR=/tmp
for cfg in "1:32:0" "1:32:1" "0:32:0" "0:32:1"; do
  kc=${cfg%%:*}; rest=${cfg#*:}; seed=${rest%%:*}; su=${rest#*:}
  MV2AMD_P2P_KERNEL_COPY=$kc DIAG_SYNC_UPLOAD=$su timeout -k 10 300 python -u tools/ringsoak_diag.py 12 4 250 $seed > $O/r_${kc}_${seed}_${su}.json 2> $O/r_${kc}_${seed}_${su}.err || { tail -30 $O/r_${kc}_${seed}_${su}.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/r_${kc}_${seed}_${su}.json')); print('kcopy',d['env_p2p'],'sync',d['sync_upload'],'wrong per rank',[r[0] for r in d['per_rank']], 'first', d['per_rank'][0][2:9])"
done
