set -o pipefail
# Round 5, pass aj: the r05ai diagnosis after the fix (intra-node unexpected payloads kept in device
# memory; every delivery of a received payload complete before its receive is; the point-to-point
# completion word trusted only for passes made of copy kernels alone)
O=gpurun_out/r05aj
mkdir -p $O
export TMPDIR=/tmp
for kc in 1 0; do
  MV2AMD_P2P_KERNEL_COPY=$kc timeout -k 10 300 python -u tools/ringsoak_diag.py 12 4 250 32 > $O/r_$kc.json 2> $O/r_$kc.err || { tail -30 $O/r_$kc.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/r_$kc.json')); pr=d['per_rank']
print('kcopy', d['env_p2p'], 'wrong', [r[0] for r in pr], 'calls with unexpected', [r[3] for r in pr])
for r in (0, 4, 8):
    det = pr[r][4:]
    print(' rank', r, 'wrong calls (call, op, count, nbad, first, last, unexpected delta):', [det[i:i+7] for i in range(0, len(det), 7)][:5])
"
done
