set -o pipefail
# MV2_* selection knobs (ring on/off and threshold, skip-table threshold, reduce-scatter ring threshold): full GPU tests + smoke().
O=gpurun_out/r01v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
