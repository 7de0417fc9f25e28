#!/bin/bash
set -o pipefail
# Round 6, pass c: the library-free probe (tools/diag/nshare_probe) with the copy engines off
# (HSA_ENABLE_SDMA=0: hipMemcpy runs blit kernels on the compute queues), the setting under which the
# library's 12-process soak went from 3-13 to 35-86 wrong calls per rank (r06b); 8 processes as the
# control; then the library's 12 = 3 x 4 soak once more with the XCD-checked completion word
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
probe() {  # tag nprocs iters mode spin_us
  local tag=$1; shift
  echo "== $tag: $* $(date +%T)"
  HSA_ENABLE_SDMA=0 timeout -k 10 240 tools/diag/nshare_probe "$@" > $O/$tag.jsonl 2> $O/$tag.err
  local rc=$?
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/$tag.jsonl') if '\"rank\"' in l]
print('$tag', 'rc', $rc, 'procs', len(r), 'secs', max([x['secs'] for x in r] or [0]),
      'pre', [x['pre']['words'] for x in r], 'post_P', [x['post_P']['words'] for x in r],
      'post_R', [x['post_R']['words'] for x in r], 'slots', [x['slots']['words'] for x in r],
      'distinct_va_P', len(set(x['va_P'] for x in r)))
" | tee -a $O/summary.txt
  return $rc
}
probe s8_ipc_spin 8 300 3 200 && probe s12_ipc_spin 12 300 3 200 && probe s12_chunked 12 300 7 200 && \
probe s9_ipc_spin 9 300 3 200 && probe s12_plain 12 300 0 0 || exit 1
run() {  # tag n ppn calls [env...]
  local tag=$1 n=$2 ppn=$3 calls=$4; shift 4
  echo "== $tag $(date +%T)"
  env "$@" DIAG_DETAIL=2 DIAG_CHECK_SB=1 timeout -k 10 300 python -u tools/ringsoak_diag.py $n $ppn $calls 32 $O/$tag > $O/$tag.json 2> $O/$tag.err || { tail -30 $O/$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$tag.json')); pr=d['per_rank']
print('$tag ($n ranks, $ppn per node, $calls calls):', 'rcs', d['rcs'], 'wrong', [r[0] if r else None for r in pr], 'sb before', [r[3] if r else None for r in pr], 'sb after', [r[4] if r else None for r in pr])
" | tee -a $O/summary.txt
  grep -l "workgroups of one group ran on several XCDs\|without raising its completion word" $O/${tag}_rank*.log | tee -a $O/summary.txt || true
}
run n12 12 4 400
