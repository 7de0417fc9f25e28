#!/bin/bash
set -o pipefail
# Round 6, pass at: the in-tree library as build() leaves it at the round's end -- smoke, the
# Reduce_local tests, the 8-rank collectives and soak, the N = 1 line
O=gpurun_out/r06at
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_reduce_local.py "tests/test_gpu_collectives_mp.py::test_collectives_multiprocess[8-default]" "tests/test_gpu_collectives_mp.py::test_soak_thousands_of_calls[8-5000-13-env2-None]" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1]); print('N=1', d['value'], d['roofline']['frac'], d['extra']['reduce_local_8B_latency_us']['us'])"
