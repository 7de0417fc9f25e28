"""Stream-ordered 8-byte allreduce loop (MPIX_Allreduce_enqueue) next to the blocking loop, for
kernel traces: python -m mvapich2_amd.mv2run -n 2 --share-gpu python tools/enqueue_probe.py"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402

W = 0x44000000
L = m.lib()
m.check(L.MPI_Init(None, None), "init")
F, SUM = TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]
s8, r8 = m.DeviceBuffer(8), m.DeviceBuffer(8)
s8.upload(np.ones(2, dtype=np.float32))
hip = ctypes.CDLL("libamdhip64.so")
st = ctypes.c_void_p()
hip.hipStreamCreate(ctypes.byref(st))
iters = int(os.environ.get("PROBE_ITERS", "200"))
for mode in ("blocking", "enqueue", "blocking", "enqueue"):
    L.MPI_Barrier(W)
    t0 = time.perf_counter()
    for _ in range(iters):
        if mode == "blocking":
            m.check(L.MPI_Allreduce(s8.ptr, r8.ptr, 2, F, SUM, W), "ar")
        else:
            m.check(L.MPIX_Allreduce_enqueue(s8.ptr, r8.ptr, 2, F, SUM, W, st), "enq")
    hip.hipStreamSynchronize(st)
    L.mv2h_device_synchronize()
    t = (time.perf_counter() - t0) / iters
    if m.lib().mv2h_rank() == 0:
        print(f"{mode}: {t * 1e6:.2f} us per call", flush=True)
hip.hipStreamDestroy(st)
L.MPI_Finalize()
