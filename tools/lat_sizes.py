"""Small-message collective latency probe (LAT_COLL = allreduce | reduce_scatter_block | bcast) (fp32 SUM, device buffers): per size, the algorithm the
selection picks, the OSU-loop wall time per call (barrier before every call, as osu_coll does)
and the kernel time from HIP events on the library's stream.  Run under mv2run, e.g.
    python -m mvapich2_amd.mv2run -n 2 --share-gpu python tools/lat_sizes.py
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402


def main():
    L = m.lib()
    m.check(L.MPI_Init(None, None), "MPI_Init")
    world = 0x44000000
    rank, size = L.mv2h_rank(), L.mv2h_size()
    F32, SUM = TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]
    sizes = [int(s) for s in os.environ.get("LAT_SIZES", "8,512,2048,4096,8192,16384,65536,262144").split(",")]
    iters = int(os.environ.get("LAT_ITERS", "2000"))
    sb, rb = m.DeviceBuffer(max(sizes)), m.DeviceBuffer(max(sizes))
    for sz in sizes:
        count = max(1, sz // 4)
        sb.upload(np.full(count, 1.0 + rank, np.float32))
        coll = os.environ.get("LAT_COLL", "allreduce")
        if coll == "allreduce":
            algo, inner, _, progs, blk = m.plan("allreduce", size, rank, F32, count)
            call = lambda: L.MPI_Allreduce(sb.ptr, rb.ptr, count, F32, SUM, world)  # noqa: E731
        elif coll == "reduce_scatter_block":
            count = max(size, count - count % size)
            sb.upload(np.full(count, 1.0 + rank, np.float32))
            algo, inner, progs = -1, 0, []
            call = lambda: L.MPI_Reduce_scatter_block(sb.ptr, rb.ptr, count // size, F32, SUM, world)  # noqa: E731
        else:
            sb.upload(np.full(count, 1.0 + size * (size + 1) / 2 - 1.0, np.float32))
            algo, inner, progs = -1, 0, []
            call = lambda: L.MPI_Bcast(sb.ptr if rank == 0 else rb.ptr, count, F32, 0, world)  # noqa: E731
            if rank == 0:
                rb.upload(np.full(count, size * (size + 1) / 2, np.float32))
        for _ in range(200):
            m.check(call(), "warmup")
        tot = 0.0
        for _ in range(iters):
            L.MPI_Barrier(world)
            t0 = time.perf_counter()
            m.check(call(), "call")
            tot += time.perf_counter() - t0
        L.mv2h_timing_enable(1)
        kms = []
        for _ in range(iters // 4):
            L.MPI_Barrier(world)
            m.check(call(), "call")
            kms.append(L.mv2h_last_kernel_ms())
        L.mv2h_timing_enable(0)
        got = rb.download(np.float32, count=count if coll == "allreduce" or coll == "bcast" else count // size)
        ok = bool(np.all(got == np.float32(size * (size + 1) / 2)))
        if rank == 0:
            print(f"{sz:>8} B  algo {algo} inner {inner} nprog {len(progs)}  wall {tot / iters * 1e6:7.2f} us  "
                  f"kernel {np.mean(kms) * 1e3:7.2f} us (p50 {np.median(kms) * 1e3:6.2f})  ok={ok}", flush=True)
    m.check(L.MPI_Finalize(), "MPI_Finalize")


if __name__ == "__main__":
    main()
