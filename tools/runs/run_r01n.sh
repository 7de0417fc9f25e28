set -o pipefail
# pipe geometry probe: 8 and 4 ranks sharing one GPU, MV2AMD_PIPE_SUB 64/32/16 KiB
O=gpurun_out/r01n
mkdir -p $O
for n in 8 4; do
for sub in 65536 32768 16384; do
  MV2AMD_PIPE_SUB=$sub timeout -k 10 200 python -m mvapich2_amd.mv2run -n $n --share-gpu --timeout 190 python -u bench.py --gpus $n --steps 8 --warmup 2 --lat-iters 50 --rccl 0 > $O/b${n}_$sub.json 2> $O/b${n}_$sub.err || { tail -5 $O/b${n}_$sub.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b${n}_$sub.json')); e=d['extra']; print($n, $sub, d['value'], d['roofline']['kernel_ms'], e['reduce_scatter_f32_sum']['busbw_GBps'], e['allgather_char']['busbw_GBps'], e['bcast_char']['busbw_GBps'], d['config']['correct'])"
done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_p2p_mp.py -x -q --timeout 150 --timeout-method thread > $O/p2p.log 2>&1; tail -2 $O/p2p.log
