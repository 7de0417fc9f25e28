set -o pipefail
# Round 3, pass q: host cost of stream-idle queries vs a kernel launch (small-message floor analysis);
# the N=1 bench line with its new 8-byte Reduce_local latency field.
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 120 ./tools/query_probe > $O/query_probe.txt 2>&1 || { cat $O/query_probe.txt; exit 1; }
cat $O/query_probe.txt
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_n1.json')); print(d['value'], d['extra']['reduce_local_8B_latency_us'])"
