set -o pipefail
O=gpurun_out/r01e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 tools/osu/osu_coll -c allreduce -m 1048576:268435456 -i 20 -x 5 -v > $O/ar_$name.txt 2>&1 || { tail $O/ar_$name.txt; exit 1; }
  echo "== $name"; tail -n 3 $O/ar_$name.txt
}
run light MV2AMD_LIGHT_RELEASE=1
run full MV2AMD_LIGHT_RELEASE=0
run g64 MV2AMD_PIPE_GRID=64
run g32 MV2AMD_PIPE_GRID=32
run sub16k MV2AMD_PIPE_SUB=16384
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 4 --share-gpu --timeout 190 tools/osu/osu_coll -c allreduce -m 1048576:268435456 -i 20 -x 5 -v > $O/ar_4share.txt 2>&1; tail -n 3 $O/ar_4share.txt
