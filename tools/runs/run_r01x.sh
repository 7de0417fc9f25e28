set -o pipefail
# Small-message shortcut ahead of the ring wrapper (knob runs incl. ring threshold 0): multi-process GPU collectives + smoke.
O=gpurun_out/r01x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
