set -o pipefail
O=gpurun_out/r02m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_collectives_mp.py tests/test_gpu_reduce_local.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 5 60 ./tools/launch_probe2 mvapich2_amd/lib/libmpi.so > $O/launch_probe.txt 2>&1 || { cat $O/launch_probe.txt; exit 1; }
cat $O/launch_probe.txt
