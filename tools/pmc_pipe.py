"""One rank of a rocprofv3 --pmc pass over the pipelined allreduce kernel
(k_pipe PIPE_AR): six MPI_Allreduce fp32 SUM calls of 64 MiB.  Launch every
rank under its own rocprofv3 from the shell (RANK / WORLD_SIZE / LOCAL_RANK /
MV2AMD_JOBID in the environment)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402

L = m.lib()
m.check(L.MPI_Init(None, None), "MPI_Init")
rank = int(os.environ.get("RANK", "0"))
nbytes = int(os.environ.get("PMC_BYTES", str(64 << 20)))
n = nbytes // 4
a, b = m.DeviceBuffer(nbytes), m.DeviceBuffer(nbytes)
a.upload(np.random.default_rng(rank).uniform(-1, 1, n).astype(np.float32))
for _ in range(6):
    m.check(L.MPI_Allreduce(a.ptr, b.ptr, n, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"], 0x44000000), "MPI_Allreduce")
L.MPI_Barrier(0x44000000)
cfg_out = os.environ.get("PMC_CONFIG_OUT")
if cfg_out and rank == 0:  # the configuration bench.py matches a pass against (pipe_traffic_for)
    import json
    json.dump({"ranks": int(os.environ.get("WORLD_SIZE", "1")), "nshare": m.info("nshare"),
               "pipe_grid": m.info("pipe_grid"), "pipe_sub": m.info("pipe_sub"), "pipe_rnt": m.info("pipe_rnt"),
               "bytes": nbytes}, open(cfg_out, "w"))
L.MPI_Finalize()
print("done", rank)
