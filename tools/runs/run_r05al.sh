set -o pipefail
# Round 5, pass al: r05ak with 64 KiB block hashes: which blocks of the operand differ at the leader
# rank's operand and what the node leader holds of it after the gather (seed 32, which went wrong
# from call 180 in r05ae / r05ai / r05aj)
O=gpurun_out/r05al
mkdir -p $O
export TMPDIR=/tmp
MV2AMD_DEBUG_GATHER=1 timeout -k 10 400 python -u tools/ringsoak_diag.py 12 4 250 32 $O/w > $O/r.json 2> $O/r.err || { tail -30 $O/r.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r.json')); pr=d['per_rank']
print('wrong', [r[0] for r in pr])
det = pr[0][4:]; print('rank 0 wrong calls', [det[i:i+7] for i in range(0, len(det), 7)][:6])
"
cat $O/w_rank*.log | grep -c "debug gather" || true
cat $O/w_rank*.log | grep "debug gather" | head -20 || true
