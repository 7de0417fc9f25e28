"""§8(f) rank 1 and 3: device point-to-point (MPI_Send/Recv/Sendrecv/Isend/
Irecv over the per-pair IPC channels) and nonblocking collectives
(MPI_Iallreduce/Ibcast/Ibarrier + Wait/Test/Waitall), one process per rank,
ranks sharing the box's GPU, on one node and across emulated nodes.  Exact checks run inside each rank
(tests/mp_p2p_worker.py)."""
import os
import subprocess
import sys
import uuid

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# MV2AMD_TEST_P2P_EXTRA="16x4,..." adds shapes
_EXTRA = [tuple(int(v) for v in s.split("x")) for s in os.environ.get("MV2AMD_TEST_P2P_EXTRA", "").split(",") if s]


# at most 8 processes on the one GPU (DESIGN.md §5 "Ranks per GPU"): 8 x 1 puts every pair but none
# on the rank mesh, 2 x 4 mixes both transports
@pytest.mark.parametrize("n,ppn", [(2, 2), (3, 3), (8, 8), (4, 2), (3, 1), (6, 3), (8, 4), (8, 1)] + _EXTRA)
def test_p2p_and_nonblocking_collectives(n, ppn):
    """ppn < n: emulated nodes (node-major ranks); messages between nodes travel the rank mesh
    (runtime/internode.cpp mesh_setup, runtime/p2p.cpp net_progress) under the same matching"""
    jobid = "p" + uuid.uuid4().hex[:12]
    boot = {}
    if ppn < n:
        import socket
        so = socket.socket()
        so.bind(("127.0.0.1", 0))
        boot = {"MV2AMD_BOOT_ADDR": "127.0.0.1", "MV2AMD_BOOT_PORT": str(so.getsockname()[1]), "MV2AMD_NSHARE": str(n)}
        so.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r % ppn), LOCAL_WORLD_SIZE=str(ppn),
                   MV2AMD_JOBID=jobid, MV2AMD_TIMEOUT_S="30", MV2AMD_DEVICE="0", MV2AMD_ERR_VERBOSE="1", **boot)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_p2p_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=150)
            logs.append(o.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    bad = [r for r, p in enumerate(procs) if p.returncode != 0]

    def last_step(log):
        steps = [ln for ln in log.splitlines() if " step " in ln and ln.startswith("rank ")]
        return steps[-1].split(" step ")[1] if steps else "-"
    assert not bad, "ranks " + ", ".join(f"{r} (rc {procs[r].returncode})" for r in bad) + " failed; last step per rank: " + \
        " ".join(f"{r}:{last_step(lg)}" for r, lg in enumerate(logs)) + "\n" + \
        "\n".join(f"--- rank {r}:\n{logs[r][-1500:]}" for r in bad)
