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


def _mn_worker(rank, size, ppn, jobid, port, counter, iters, q):
    try:
        os.environ.update(MV2AMD_CONTROL_PLANE_ONLY="1", MV2AMD_JOBID=jobid, RANK=str(rank), WORLD_SIZE=str(size),
                          LOCAL_RANK=str(rank % ppn), LOCAL_WORLD_SIZE=str(ppn), MV2AMD_BOOT_ADDR="127.0.0.1",
                          MV2AMD_BOOT_PORT=str(port), MV2AMD_TIMEOUT_S="60")
        import mvapich2_amd as m
        L = m.lib()
        assert L.mv2h_init() == 0
        assert L.mv2h_rank() == rank and L.mv2h_size() == size and L.mv2h_local_rank() == rank % ppn
        assert m.info("nnodes") == size // ppn and m.info("node") == rank // ppn
        for k in range(iters):
            with counter.get_lock():
                counter.value += 1
            assert L.mv2h_barrier() == 0
            assert counter.value >= size * (k + 1), (rank, k, counter.value)
        assert L.mv2h_finalize() == 0
        q.put((rank, "ok"))
    except BaseException as e:
        q.put((rank, repr(e)))


@pytest.mark.parametrize("size,ppn", [(4, 2), (6, 2), (3, 1), (8, 4)])
def test_multinode_bootstrap_and_global_barrier(size, ppn):
    """Several nodes emulated on one host: every node gets its own
    control segment, the node leaders rendezvous at MV2AMD_BOOT_ADDR:PORT and link over TCP
    (runtime/internode.cpp); MPI_Barrier = node barrier + leaders' dissemination barrier + node
    barrier, so no rank passes barrier k before every rank of every node has reached it."""
    import socket
    ctx = mp.get_context("fork")
    counter = ctx.Value("i", 0)
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    jobid = "n" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_mn_worker, args=(r, size, ppn, jobid, port, counter, 50, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res
    assert counter.value == 50 * size


def test_multinode_needs_node_major_ranks():
    ctx = mp.get_context("fork")
    q = ctx.Queue()

    def w(q):
        # rank 1 claiming local rank 0 of 2: not numbered node-major
        os.environ.update(MV2AMD_CONTROL_PLANE_ONLY="1", RANK="1", WORLD_SIZE="4", LOCAL_RANK="0",
                          LOCAL_WORLD_SIZE="2", MV2AMD_JOBID="t" + uuid.uuid4().hex[:8])
        import mvapich2_amd as m
        q.put(m.lib().mv2h_init())

    p = ctx.Process(target=w, args=(q,))
    p.start()
    rc = q.get(timeout=60)
    p.join()
    assert rc == 44  # MPI_ERR_UNSUPPORTED_OPERATION


def test_mv2run_node_emulation_environment(tmp_path):
    """mv2run --nodes K: node-major local ranks, one boot port for the leaders, the GPU-sharing
    hint when --share-gpu is given (mvapich2_amd/mv2run.py)."""
    import json
    import subprocess
    import sys
    out = tmp_path / "env"
    out.mkdir()
    child = ("import json, os, sys; k = ['RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'LOCAL_WORLD_SIZE', "
             "'MV2_COMM_WORLD_LOCAL_RANK', 'MV2AMD_BOOT_PORT', 'MV2AMD_NSHARE', 'MV2AMD_DEVICE', 'MV2AMD_JOBID']; "
             "open(os.path.join(sys.argv[1], os.environ['RANK']), 'w').write(json.dumps({x: os.environ.get(x) for x in k}))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rc = subprocess.run([sys.executable, "-m", "mvapich2_amd.mv2run", "-n", "6", "--nodes", "3", "--share-gpu",
                         "--timeout", "60", sys.executable, "-c", child, str(out)], cwd=root, timeout=120).returncode
    assert rc == 0
    envs = [json.loads((out / str(r)).read_text()) for r in range(6)]
    for r, e in enumerate(envs):
        assert e["RANK"] == str(r) and e["WORLD_SIZE"] == "6"
        assert e["LOCAL_RANK"] == e["MV2_COMM_WORLD_LOCAL_RANK"] == str(r % 2) and e["LOCAL_WORLD_SIZE"] == "2"
        assert e["MV2AMD_NSHARE"] == "6" and e["MV2AMD_DEVICE"] == "0"
    assert len({e["MV2AMD_BOOT_PORT"] for e in envs}) == 1 and envs[0]["MV2AMD_BOOT_PORT"]
    assert len({e["MV2AMD_JOBID"] for e in envs}) == 1


def _mn_knob_worker(rank, size, ppn, jobid, port, q):
    try:
        os.environ.update(MV2AMD_CONTROL_PLANE_ONLY="1", MV2AMD_JOBID=jobid, RANK=str(rank), WORLD_SIZE=str(size),
                          LOCAL_RANK=str(rank % ppn), LOCAL_WORLD_SIZE=str(ppn), MV2AMD_BOOT_ADDR="127.0.0.1",
                          MV2AMD_BOOT_PORT=str(port), MV2AMD_TIMEOUT_S="30")
        if rank // ppn == 1:  # the second node's ranks agree among themselves, not with node 0
            os.environ["MV2_ALLRED_USE_RING"] = "0"
        import mvapich2_amd as m
        q.put((rank, m.lib().mv2h_init()))
    except BaseException as e:
        q.put((rank, repr(e)))


def test_multinode_knob_mismatch_fails_every_rank():
    """Nodes started with different MV2_* selection knobs would pair different schedules: node 0's
    leader refuses the job at the rendezvous (runtime/internode.cpp Hello.knob_hash) and every rank
    of every node fails MPI_Init instead of hanging or computing garbage later."""
    import socket
    size, ppn = 4, 2
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    jobid = "k" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_mn_knob_worker, args=(r, size, ppn, jobid, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v not in (0, None) and not isinstance(v, str) for v in res.values()), res
