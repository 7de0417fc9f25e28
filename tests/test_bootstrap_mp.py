"""COMM_WORLD bootstrap over the /dev/shm control plane, multi-process on CPU
(MV2AMD_CONTROL_PLANE_ONLY=1: no GPU is touched).  Covers rank discovery from
the torchrun / MV2 environment variables and the host barrier used for the
per-call buffer-descriptor exchange of the device collectives."""
import multiprocessing as mp
import os
import uuid

import pytest


def _worker(rank, size, jobid, counter, iters, env_style, q):
    try:
        os.environ["MV2AMD_CONTROL_PLANE_ONLY"] = "1"
        os.environ["MV2AMD_JOBID"] = jobid
        if env_style == "torchrun":
            os.environ.update(RANK=str(rank), WORLD_SIZE=str(size), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(size))
        else:
            os.environ.update(MV2_COMM_WORLD_RANK=str(rank), MV2_COMM_WORLD_SIZE=str(size),
                              MV2_COMM_WORLD_LOCAL_RANK=str(rank))
        import mvapich2_amd as m
        L = m.lib()
        assert L.mv2h_init() == 0
        assert L.mv2h_rank() == rank and L.mv2h_size() == size
        for k in range(iters):
            with counter.get_lock():
                counter.value += 1
            assert L.mv2h_barrier() == 0
            assert counter.value >= size * (k + 1), (rank, k, counter.value)
        assert L.mv2h_finalize() == 0
        q.put((rank, "ok"))
    except BaseException as e:  # report to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("size,env_style", [(2, "torchrun"), (4, "mv2"), (8, "torchrun")])
def test_shm_barrier(size, env_style):
    ctx = mp.get_context("fork")
    counter = ctx.Value("i", 0)
    q = ctx.Queue()
    jobid = "t" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_worker, args=(r, size, jobid, counter, 200, env_style, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res
    assert counter.value == 200 * size
    assert not os.path.exists("/dev/shm/mv2amd." + jobid)  # rank 0 unlinked the segment


def test_multinode_launch_is_rejected():
    ctx = mp.get_context("fork")
    q = ctx.Queue()

    def w(q):
        os.environ.update(MV2AMD_CONTROL_PLANE_ONLY="1", RANK="0", WORLD_SIZE="4", LOCAL_WORLD_SIZE="2",
                          MV2AMD_JOBID="t" + uuid.uuid4().hex[:8])
        import mvapich2_amd as m
        q.put(m.lib().mv2h_init())

    p = ctx.Process(target=w, args=(q,))
    p.start()
    rc = q.get(timeout=60)
    p.join()
    assert rc == 44  # MPI_ERR_UNSUPPORTED_OPERATION
