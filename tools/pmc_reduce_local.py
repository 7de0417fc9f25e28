"""Short program for rocprofv3 --pmc passes: six MPI_Reduce_local fp32 SUM
calls on 256 MiB random device operands (the bench's N=1 workload)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402

L = m.lib()
n = 64 << 20
rng = np.random.default_rng(0x5EED)
a, b = m.DeviceBuffer(n * 4), m.DeviceBuffer(n * 4)
a.upload(rng.uniform(-1, 1, n).astype(np.float32))
b.upload(rng.uniform(-1, 1, n).astype(np.float32))
for _ in range(6):
    m.check(L.MPI_Reduce_local(a.ptr, b.ptr, n, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]), "MPI_Reduce_local")
print("done")
