set -o pipefail
# Round 5, pass ar: does a rank's send buffer change during the multi-node ring allreduce?  The
# soak reads its operand back before and after every call (seed 32, 12 = 3 x 4), current library,
# then the round-4 one
O=gpurun_out/r05ar
mkdir -p $O
export TMPDIR=/tmp
DIAG_DETAIL=2 DIAG_CHECK_SB=1 timeout -k 10 500 python -u tools/ringsoak_diag.py 12 4 250 32 $O/new > $O/new.json 2> $O/new.err || { tail -30 $O/new.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/new.json')); pr=d['per_rank']
print('current: wrong', [r[0] for r in pr], 'sb wrong before', [r[3] for r in pr], 'sb changed after', [r[4] for r in pr])
for r, x in enumerate(pr):
    if x[5:]: print('  rank', r, 'sb changes (call, n, first, last, delta):', [x[5:][i:i+5] for i in range(0, len(x[5:]), 5)][:4])
"
MV2AMD_LIBMPI=$PWD/tools/diag/libmpi_r04.so DIAG_DETAIL=2 DIAG_CHECK_SB=1 timeout -k 10 500 python -u tools/ringsoak_diag.py 12 4 250 32 $O/old > $O/old.json 2> $O/old.err || { tail -30 $O/old.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/old.json')); pr=d['per_rank']
print('round 4: wrong', [r[0] for r in pr], 'sb wrong before', [r[3] for r in pr], 'sb changed after', [r[4] for r in pr])
for r, x in enumerate(pr):
    if x[5:]: print('  rank', r, 'sb changes (call, n, first, last, delta):', [x[5:][i:i+5] for i in range(0, len(x[5:]), 5)][:4])
"
