set -o pipefail
# Round 5, pass s: a long soak — 100k / 60k / 30k mixed calls at 2 / 4 / 8 shared ranks, every
# result checked against its closed form (MV2AMD_SOAK_CALLS); one pytest run per rank count so
# that each prints before the next starts
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
for spec in "2-100000:2-16000-11-env0-None" "4-60000:4-10000-12-env1-None" "8-30000:8-5000-13-env2-None"; do
  calls=${spec%%:*}; calls=${calls#*-}; id=${spec#*:}
  MV2AMD_SOAK_CALLS=$calls timeout -k 10 420 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread \
    "tests/test_gpu_collectives_mp.py::test_soak_thousands_of_calls[$id]" --durations=1 > $O/soak_$id.log 2>&1 \
    || { echo "soak $id failed"; tail -60 $O/soak_$id.log; exit 1; }
  grep -E "passed|call " $O/soak_$id.log
done
