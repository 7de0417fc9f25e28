set -o pipefail
# Round 5, pass as: does the multi-node ring corruption depend on the number of processes sharing
# the one GPU?  The amdgpu scheduler parameters, then the same ring soak (seed 32) at 6 = 3 x 2,
# 8 = 2 x 4, 9 = 3 x 3 and 12 = 3 x 4 ranks
O=gpurun_out/r05as
mkdir -p $O
export TMPDIR=/tmp
for f in hws_max_conc_proc sched_policy mes noretry vm_fragment_size hws_gws_support; do
  echo "$f=$(cat /sys/module/amdgpu/parameters/$f 2>/dev/null)"; done | tee $O/params.txt
for cfg in "6 2" "8 4" "9 3" "12 4"; do
  set -- $cfg
  DIAG_DETAIL=2 DIAG_CHECK_SB=1 timeout -k 10 300 python -u tools/ringsoak_diag.py $1 $2 200 32 $O/n$1 > $O/n$1.json 2> $O/n$1.err || { tail -30 $O/n$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/n$1.json')); pr=d['per_rank']
print('$1 ranks x $2:', 'rcs', d['rcs'], 'wrong', [r[0] if r else None for r in pr], 'sb before', [r[3] if r else None for r in pr], 'sb after', [r[4] if r else None for r in pr])
for r, x in enumerate(pr):
    if x[5:]: print('  rank', r, 'sb changes (call, n, first, last, delta):', [x[5:][i:i+5] for i in range(0, len(x[5:]), 5)][:4])
" | tee -a $O/summary.txt
done
