set -o pipefail
# Round 5, pass ao: the gather check with each sender's operand hashed before and after its send, and the
# leader's own operand in G (copies via hipMemcpy) checked too
# copy kernels and copy engines, seed 32
O=gpurun_out/r05ao
mkdir -p $O
export TMPDIR=/tmp
for kc in 1 0; do
  MV2AMD_P2P_KERNEL_COPY=$kc MV2AMD_DEBUG_GATHER=1 timeout -k 10 400 python -u tools/ringsoak_diag.py 12 4 250 32 $O/w$kc > $O/r$kc.json 2> $O/r$kc.err || { tail -30 $O/r$kc.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/r$kc.json')); pr=d['per_rank']
print('kcopy $kc wrong', [r[0] for r in pr])
det = pr[0][4:]; print('rank 0 wrong calls', [det[i:i+7] for i in range(0, len(det), 7)][:4])
"
  cat $O/w${kc}_rank*.log | grep -c "debug gather" || true
  cat $O/w${kc}_rank*.log | grep "debug gather" | head -6 || true
done
