set -o pipefail
# Round 5, pass aq: bisect the multi-node ring mismatch: the round-4 library (6cbd434, built from
# its own sources into tools/diag/libmpi_r04.so) against the current one on the same box, seed 32,
# 250 calls at 12 = 3 x 4
O=gpurun_out/r05aq
mkdir -p $O
export TMPDIR=/tmp
MV2AMD_LIBMPI=$PWD/tools/diag/libmpi_r04.so DIAG_DETAIL=0 timeout -k 10 400 python -u tools/ringsoak_diag.py 12 4 250 32 $O/old > $O/old.json 2> $O/old.err || { tail -30 $O/old.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/old.json')); print('round 4 lib wrong', [r[0] for r in d['per_rank']], 'first', [r[2] for r in d['per_rank']])"
DIAG_DETAIL=0 timeout -k 10 400 python -u tools/ringsoak_diag.py 12 4 250 32 $O/new > $O/new.json 2> $O/new.err || { tail -30 $O/new.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/new.json')); print('current lib wrong', [r[0] for r in d['per_rank']], 'first', [r[2] for r in d['per_rank']])"
