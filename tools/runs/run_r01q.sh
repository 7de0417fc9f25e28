set -o pipefail
# 2-rank shared-GPU bench, three repeats (noise estimate)
O=gpurun_out/r01q
mkdir -p $O
for i in 1 2 3; do
timeout -k 10 200 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 190 python -u bench.py --gpus 2 --steps 10 --warmup 3 --lat-iters 100 --rccl 0 > $O/b2_$i.json 2> $O/b2_$i.err || { tail -5 $O/b2_$i.err; exit 1; }
python -c "import json; d=json.load(open('$O/b2_$i.json')); e=d['extra']; print(d['value'], e['reduce_scatter_f32_sum']['busbw_GBps'], e['allgather_char']['busbw_GBps'], e['bcast_char']['busbw_GBps'], d['config']['correct'])"
done
