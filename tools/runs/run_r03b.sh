set -o pipefail
# Round 3, pass b: the reworked user-op path, MPI_Testall, multi-level topology on the device,
# multi-node flat nonblocking schedules, pack/unpack host overhead probe, 8-rank shared bench.
O=gpurun_out/r03b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/osu/pack_overhead > $O/pack_overhead.json 2> $O/pack_overhead.err || { tail -5 $O/pack_overhead.err; exit 1; }
cat $O/pack_overhead.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_p2p_mp.py \
  "tests/test_gpu_collectives_mp.py::test_user_op_on_strided_vector_operand" \
  "tests/test_gpu_collectives_mp.py::test_gpu_topology_levels" \
  "tests/test_gpu_collectives_mp.py::test_collectives_multiprocess[3-default]" \
  tests/test_gpu_multinode_mp.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -80 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
timeout -k 10 300 python -m mvapich2_amd.mv2run -n 8 --share-gpu --timeout 290 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lat-iters 200 > $O/bench_8share.json 2> $O/bench_8share.err || { tail -20 $O/bench_8share.err; exit 1; }
cat $O/bench_8share.json
