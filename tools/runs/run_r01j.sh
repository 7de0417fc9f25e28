set -o pipefail
# New Reduce_local shape (nt loads + plain stores, 512x2, full grid) +
# two-level completion counters: sync probe, PMC traffic passes, full check.
O=gpurun_out/r01j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/sync_probe.py > $O/sync.txt 2>&1 || exit 1
cat $O/sync.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o f -- python3 tools/pmc_reduce_local.py > $O/pmc_f.log 2>&1 || { tail -5 $O/pmc_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o w -- python3 tools/pmc_reduce_local.py > $O/pmc_w.log 2>&1 || { tail -5 $O/pmc_w.log; exit 1; }
F=$(find $O/pmc_f -name '*counter_collection.csv' | head -1)
W=$(find $O/pmc_w -name '*counter_collection.csv' | head -1)
python tools/pmc_summary.py "$F" "$W" "k_reduce_local<mv2::R<2, 8, void>, 2>" $O/pmc_reduce_local.json 805306368 && cat $O/pmc_reduce_local.json
bash tools/gpu_check.sh r01j || exit 1
