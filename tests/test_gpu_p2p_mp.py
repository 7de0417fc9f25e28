"""§8(f) rank 1 and 3: device point-to-point (MPI_Send/Recv/Sendrecv/Isend/
Irecv over the per-pair IPC channels) and nonblocking collectives
(MPI_Iallreduce/Ibcast/Ibarrier + Wait/Test/Waitall), one process per rank,
ranks sharing the box's GPU.  Exact checks run inside each rank
(tests/mp_p2p_worker.py)."""
import os
import subprocess
import sys
import uuid

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3, 8])
def test_p2p_and_nonblocking_collectives(n):
    jobid = "p" + uuid.uuid4().hex[:12]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MV2AMD_JOBID=jobid, MV2AMD_TIMEOUT_S="30", MV2AMD_DEVICE="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_p2p_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=110)
            logs.append(o.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-3000:]}"
