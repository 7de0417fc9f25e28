"""Short program for rocprofv3 passes over the device pack / unpack kernels on
BASELINE configs[4]'s strided operand: MPI_Type_vector(N, 4, 8, MPI_FLOAT)
with N = 8 Mi blocks (256 MiB strided span, 128 MiB packed), six MPI_Pack and
six MPI_Unpack calls (PMC_MODE=pack or unpack: only those).  Algorithmic HBM
bytes per call = 2 x packed bytes."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import TYPES  # noqa: E402

L = m.lib()
m.check(L.MPI_Init(None, None), "MPI_Init")
nb = 8 << 20
vt = ctypes.c_int()
m.check(L.MPI_Type_vector(nb, 4, 8, TYPES["MPI_FLOAT"][0], ctypes.byref(vt)), "MPI_Type_vector")
m.check(L.MPI_Type_commit(ctypes.byref(vt)), "MPI_Type_commit")
span = ((nb - 1) * 8 + 4) * 4
packed = nb * 16
src = m.DeviceBuffer(span)
src.upload(np.random.default_rng(1).standard_normal(span // 4).astype(np.float32))
dst = m.DeviceBuffer(packed)
mode = os.environ.get("PMC_MODE", "both")
for _ in range(6 if mode in ("both", "pack") else 0):
    pos = ctypes.c_int(0)
    m.check(L.MPI_Pack(src.ptr, 1, vt.value, dst.ptr, packed, ctypes.byref(pos), 0x44000000), "MPI_Pack")
for _ in range(6 if mode in ("both", "unpack") else 0):
    pos = ctypes.c_int(0)
    m.check(L.MPI_Unpack(dst.ptr, packed, ctypes.byref(pos), src.ptr, 1, vt.value, 0x44000000), "MPI_Unpack")
L.mv2h_device_synchronize()
L.MPI_Finalize()
print("done")
