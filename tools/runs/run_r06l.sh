#!/bin/bash
set -o pipefail
# Round 6, pass l: Reduce_local tests with the HSA-queue path (incl. null-stream ordering and copy
# rewrites), smoke, the N = 1 line (8-byte latency via the queue; the 256 MiB kernel with the
# folded XCD check) with rocprofv3 kernel statistics
O=gpurun_out/r06l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_reduce_local.py > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc = 0 ] || { grep -B5 -A40 "Error\|FAIL" $O/pytest.log | head -100; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
cp $(find $O/prof -name '*kernel_stats*' | head -1) $O/rocprof_kernel_stats.csv && rm -rf $O/prof
python3 -c "
import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
print('N=1', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['extra']['reduce_local_8B_latency_us'], d['extra']['completion_word'], d['cpu_baseline']['value'], d['extra']['cpu_host_allreduce_8rank'].get('l3_domains_used'), d['extra']['cpu_host_allreduce_8rank'].get('latency_8B_us'))"
head -3 $O/rocprof_kernel_stats.csv | cut -c1-200
