set -o pipefail
O=gpurun_out/r02z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_reduce_n.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_pack.log 2>&1 || { tail -40 $O/pytest_pack.log; exit 1; }
tail -2 $O/pytest_pack.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['extra']['MPI_Pack/Unpack MPI_Type_vector(8Mi,4,8,MPI_FLOAT)'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
timeout -k 10 400 python -m mvapich2_amd.mv2run -n 2 --share-gpu --timeout 390 tools/osu/osu_coll -c allreduce -m 8:1073741824 -i 20 -x 5 -v > $O/osu_allreduce_2share_1GiB.txt 2>&1 || { tail $O/osu_allreduce_2share_1GiB.txt; exit 1; }
tail -12 $O/osu_allreduce_2share_1GiB.txt
