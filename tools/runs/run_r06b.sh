#!/bin/bash
set -o pipefail
# Round 6, pass b: (1) XCD placement with 12 processes at once (tools/diag/xcd_probe); (2) the
# library-free probe with many small copy-engine packets at 12 processes; (3) the library's 12 = 3 x 4
# emulated-node ring soak (tools/ringsoak_diag.py, operands read back before / after every call)
# as is, with the copy engines off (HSA_ENABLE_SDMA=0: blit kernels), with 4 hardware queues per
# process instead of the 2 the library sets for shared GPUs, and with copy-engine point-to-point
O=gpurun_out/r06b
mkdir -p $O
export TMPDIR=/tmp
pids=""
for i in $(seq 1 12); do timeout -k 10 200 tools/diag/xcd_probe 1500 > $O/xcd_$i.json 2>&1 & pids="$pids $!"; done
rc=0; for p in $pids; do wait $p || rc=1; done
cat $O/xcd_*.json | tee $O/xcd_all.txt
[ $rc = 0 ] || exit 1
timeout -k 10 240 tools/diag/nshare_probe 12 300 7 200 > $O/p12_chunked.jsonl 2> $O/p12_chunked.err || exit 1
python3 -c "
import json
r=[json.loads(l) for l in open('$O/p12_chunked.jsonl') if '\"rank\"' in l]
print('p12_chunked', [(x['pre']['words'], x['post_P']['words'], x['post_R']['words'], x['slots']['words']) for x in r])" | tee -a $O/summary.txt
run() {  # tag n ppn calls [env...]
  local tag=$1 n=$2 ppn=$3 calls=$4; shift 4
  echo "== $tag $(date +%T)"
  env "$@" DIAG_DETAIL=2 DIAG_CHECK_SB=1 timeout -k 10 300 python -u tools/ringsoak_diag.py $n $ppn $calls 32 $O/$tag > $O/$tag.json 2> $O/$tag.err || { tail -30 $O/$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/$tag.json')); pr=d['per_rank']
print('$tag ($n ranks, $ppn per node, $calls calls):', 'rcs', d['rcs'], 'wrong', [r[0] if r else None for r in pr], 'sb before', [r[3] if r else None for r in pr], 'sb after', [r[4] if r else None for r in pr])
" | tee -a $O/summary.txt
}
run n12 12 4 400 && run n12_nosdma 12 4 400 HSA_ENABLE_SDMA=0 && run n12_hwq4 12 4 400 MV2AMD_HW_QUEUES=4 && \
run n12_p2pce 12 4 400 MV2AMD_P2P_KERNEL_COPY=0
