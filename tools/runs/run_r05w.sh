set -o pipefail
# Round 5, pass w: every stream-ordered collective capturable into HIP graphs (graph lane for
# reduce-scatter / allgather / broadcast / reduce), the one-shot allgather / broadcast kernel on the
# lane's device epochs; graph, enqueue, autotune (self-test count) and soak tests
O=gpurun_out/r05w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread --durations=5 \
  tests/test_gpu_collectives_mp.py -k "graph or enqueue or autotune or soak or stream" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -150 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest.log | sed 's/.*:://' ; tail -3 $O/pytest.log
