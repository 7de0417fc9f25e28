"""Per-call overhead probe for the blocking MPI path on one MI355X:
MPI_Reduce_local wall time per call (256 MiB and 64 B operands) under each
completion-wait mode (MV2AMD_SYNC) and with/without event timing.
Usage: python tools/sync_probe.py            (spawns one child per mode)"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child():
    import mvapich2_amd as m
    from mvapich2_amd.consts import OPS, TYPES
    L = m.lib()
    F, SUM = TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]
    res = {"mode": int(os.environ.get("MV2AMD_SYNC", "0")), "rl_grid": int(os.environ.get("MV2AMD_RL_GRID", "0"))}
    for label, count, iters in (("256MiB", 64 << 20, 40), ("64B", 16, 3000)):
        a, b = m.DeviceBuffer(count * 4), m.DeviceBuffer(count * 4)
        a.upload(np.ones(count, np.float32))
        b.upload(np.zeros(count, np.float32))
        for timing in (0, 1):
            for _ in range(5):
                L.MPI_Reduce_local(a.ptr, b.ptr, count, F, SUM)
            L.mv2h_timing_enable(timing)
            ks = []
            L.mv2h_device_synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                L.MPI_Reduce_local(a.ptr, b.ptr, count, F, SUM)
                if timing:
                    ks.append(L.mv2h_last_kernel_ms())
            t = (time.perf_counter() - t0) / iters
            L.mv2h_timing_enable(0)
            res[f"{label}_t{timing}_us"] = round(t * 1e6, 2)
            if timing:
                res[f"{label}_kernel_us"] = round(float(np.mean(ks)) * 1e3, 2)
        del a, b
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
    else:
        for mode, grid in ((1, 1 << 20), (0, 1 << 20), (0, 8192), (0, 4096)):
            env = dict(os.environ, MV2AMD_SYNC=str(mode), MV2AMD_RL_GRID=str(grid))
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, timeout=120,
                               capture_output=True, text=True)
            print(r.stdout.strip() or r.stderr[-500:], flush=True)
