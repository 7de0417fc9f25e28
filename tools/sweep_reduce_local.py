#!/usr/bin/env python3
"""Sweep the Reduce_local grid size on one GPU (kernel GB/s from HIP events)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402

L = m.lib()
S = 256 << 20
for tname in ("MPI_FLOAT", "MPI_DOUBLE"):
    dt = m.np_dtype(tname)
    count = S // dt.itemsize
    a = m.DeviceBuffer(S)
    b = m.DeviceBuffer(S)
    a.upload(np.ones(count, dtype=dt))
    b.upload(np.ones(count, dtype=dt))
    for grid in (256, 512, 1024, 2048, 4096, 8192, 16384, 1 << 30):
        L.mv2h_set_tuning(b"rl_grid", grid)
        for _ in range(3):
            L.MPI_Reduce_local(a.ptr, b.ptr, count, TYPES[tname][0], OPS["MPI_SUM"])
        L.mv2h_timing_enable(1)
        ks = []
        for _ in range(10):
            L.MPI_Reduce_local(a.ptr, b.ptr, count, TYPES[tname][0], OPS["MPI_SUM"])
            ks.append(L.mv2h_last_kernel_ms())
        L.mv2h_timing_enable(0)
        ms = float(np.median(ks))
        print(f"{tname} grid={grid:>10d} kernel {ms:.4f} ms  {3 * S / ms / 1e6:.1f} GB/s", flush=True)
