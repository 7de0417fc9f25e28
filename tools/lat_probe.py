"""8-byte MPI_Allreduce latency probe (one rank; run every rank, e.g. each under
its own `rocprofv3 --kernel-trace`).  Prints per-rank wall-clock statistics of
ITERS blocking calls (fp32 SUM, count 2, device buffers) as one JSON line.
With the kernel traces of every rank (tools/lat_breakdown.py) the call splits
into: host time before the launch, kernel time waiting for the peers (launch
skew), the kernel's own work, and the return after the completion word."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402

L = m.lib()
m.check(L.MPI_Init(None, None), "MPI_Init")
rank = int(os.environ.get("RANK", "0"))
iters = int(os.environ.get("LAT_ITERS", "2000"))
count = int(os.environ.get("LAT_COUNT", "2"))
a, b = m.DeviceBuffer(max(16, count * 4)), m.DeviceBuffer(max(16, count * 4))
a.upload(np.ones(count, np.float32))
W, F, S = 0x44000000, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]
f = L.MPI_Allreduce
for _ in range(200):
    f(a.ptr, b.ptr, count, F, S, W)
L.MPI_Barrier(W)
ts = np.empty(iters)
for i in range(iters):
    t0 = time.perf_counter_ns()
    f(a.ptr, b.ptr, count, F, S, W)
    ts[i] = time.perf_counter_ns() - t0
ok = bool(np.all(b.download(np.float32, count) == float(L.mv2h_size())))
L.MPI_Barrier(W)
L.MPI_Finalize()
print(json.dumps({"rank": rank, "iters": iters, "count": count, "correct": ok,
                  "mean_us": round(ts.mean() / 1e3, 3), "p50_us": round(float(np.median(ts)) / 1e3, 3),
                  "p10_us": round(float(np.percentile(ts, 10)) / 1e3, 3),
                  "p90_us": round(float(np.percentile(ts, 90)) / 1e3, 3)}), flush=True)
