set -o pipefail
# Round 5, pass b: code-object load before / after the fatbin cut; the pooled device temporaries
# (no hipMalloc in warm derived-type calls, 64 KiB derived MPI_Bcast latency with and without);
# the whole -m gpu suite; the 2-rank line (DOUBLE_INT MAXLOC back on the wide body)
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/coload_probe.py tools/oldlib/libmpi_r04.so mvapich2_amd/lib/libmpi.so > $O/coload.jsonl 2> $O/coload.err || { tail -20 $O/coload.err; exit 1; }
cat $O/coload.jsonl
rm -f $O/record.jsonl
MV2AMD_TEST_RECORD=$PWD/$O/record.jsonl timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread tests/test_gpu_collectives_mp.py -k derived_type_calls > $O/pytest_derived.log 2>&1 || { tail -60 $O/pytest_derived.log; exit 1; }
cat $O/record.jsonl
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 480 --timeout-method thread tests > $O/pytest.log 2>&1 || { echo "tests failed"; tail -120 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_torchrun2.json 2> $O/bench_torchrun2.err || { tail -30 $O/bench_torchrun2.err; exit 1; }
grep "MPI_Init" $O/bench_torchrun2.err | head -2
