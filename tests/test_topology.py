"""Topology levels of the topology-aware shm tree (runtime/orders.cpp prog_tree, world.cpp
my_topology) against the oracle's rank-by-rank simulation of the reference's multi-level
communicators: create_intra_node_multi_level_topo_comm (create_2level_comm.c:916-986) splitting
the node by each rank's NUMA node, then socket (hwloc_bind.c:2180-2298), and one
mv2_shm_tree_reduce per level (allreduce_osu.c:2340-2361, reduce_osu.c:272-296).

CPU only: the programs are evaluated on the host with the oracle's op loop (tests/test_orders.py
eval_progs); the -m gpu test test_gpu_topology_levels runs the same orders on the device.
Topologies are synthetic: one socket, two sockets spread (rank % 2), two blocked, four NUMA
nodes, NUMA + socket levels, and random ids; the bootstrap test checks that MPI_Init publishes
every rank's ids (MV2AMD_TOPO override) to every rank."""
import ctypes
import multiprocessing as mp
import os
import uuid

import numpy as np
import pytest

import mvapich2_amd as m
from mvapich2_amd.consts import OPS, TYPES
from oracle import oracle
from tests.test_orders import allreduce_via_plan, eval_progs, wide


def topologies(n, rng):
    yield "one socket", []
    yield "two sockets spread", [[r % 2 for r in range(n)]]
    yield "two sockets blocked", [[(2 * r) // n for r in range(n)]]
    yield "four NUMA spread", [[r % 4 for r in range(n)]]
    yield "NUMA + socket", [[r % 4 for r in range(n)], [(r % 4) // 2 for r in range(n)]]
    yield "every rank alone", [list(range(n))]
    for k in range(4):
        lv = int(rng.integers(1, 3))
        yield f"random {k}", [[int(c) for c in rng.integers(0, 3, n)] for _ in range(lv)]


def set_topo(levels, n):
    flat = [c for lv in levels for c in lv]
    arr = (ctypes.c_int * max(1, len(flat)))(*flat)
    assert m.lib().mv2h_set_topology(len(levels), arr, n) == 0
    oracle.set_topology(levels, n)


@pytest.fixture(autouse=True)
def _reset_topology():
    yield
    m.lib().mv2h_set_topology(0, None, 0)
    oracle.set_topology([], 1)


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_topo_tree_levels_match_reference(n):
    rng = np.random.default_rng(4000 + n)
    for name, levels in topologies(n, rng):
        set_topo(levels, n)
        for t, op, count in (("MPI_FLOAT", "MPI_SUM", 7), ("MPI_DOUBLE", "MPI_SUM", 3), ("MPI_FLOAT", "MPI_MAX", 100)):
            h = TYPES[t][0]
            assert oracle.ALGOS[m.plan("allreduce", n, 0, h, count=count)[0]] == "topo_tree"
            xs = [wide(t, count, rng) for _ in range(n)]
            got = allreduce_via_plan(xs, n, count, t, op)
            want = oracle.allreduce_ref([x.copy() for x in xs], count, h, OPS[op])
            for r in range(n):
                assert np.array_equal(got[r], want[r]), (name, levels, t, op, r)


def test_levels_change_the_order():
    """Two sockets spread at 8 ranks: tree({0,2,4,6}) then tree of the leaders {0, 1} is another
    bracketing than the one-level degree-4 tree, and fp sums show it."""
    n, t, op, count = 8, "MPI_FLOAT", "MPI_SUM", 64
    h = TYPES[t][0]
    rng = np.random.default_rng(9)
    xs = [wide(t, count, rng) for _ in range(n)]
    set_topo([], n)
    one = allreduce_via_plan(xs, n, count, t, op)[0]
    set_topo([[r % 2 for r in range(n)]], n)
    two = allreduce_via_plan(xs, n, count, t, op)[0]
    prog = m.plan("allreduce", n, 0, h, count=count)[3][0]
    # level 0: socket 0 = ranks 0 2 4 6 (degree 4: 0 <- 2, 4, 6), socket 1 = 1 3 5 7 into 1; level 1: 0 <- 1
    assert prog == ([(0, 2), (0, 4), (0, 6), (1, 3), (1, 5), (1, 7), (0, 1)], 0), prog
    assert not np.array_equal(one, two)


@pytest.mark.parametrize("n", [4, 8])
def test_reduce_topo_levels_match_reference(n, monkeypatch):
    """MPI_Reduce's topology-aware path (MV2_USE_TOPO_AWARE_REDUCE=1) walks the same levels"""
    monkeypatch.setenv("MV2_USE_TOPO_AWARE_REDUCE", "1")
    m.lib().mv2h_knobs_reload()
    try:
        rng = np.random.default_rng(77 + n)
        k = oracle.default_knobs(use_topo_reduce=1)
        for name, levels in topologies(n, rng):
            set_topo(levels, n)
            t, op, count = "MPI_FLOAT", "MPI_SUM", 9
            h, _, _, ext = TYPES[t]
            for root in (0, n - 1):
                algo, _, _, progs, blk = m.plan("reduce", n, root, h, count=count, root=root)
                assert oracle.ALGOS[algo] == "reduce_topo", oracle.ALGOS[algo]
                xs = [wide(t, count, rng) for _ in range(n)]
                got = eval_progs(xs, progs, blk, 0, count, ext, h, OPS[op])
                want = oracle.reduce_ref([x.copy() for x in xs], count, h, OPS[op], root, knobs=k)
                assert np.array_equal(got, want), (name, levels, root)
    finally:
        monkeypatch.delenv("MV2_USE_TOPO_AWARE_REDUCE")
        m.lib().mv2h_knobs_reload()


def _boot_worker(rank, size, jobid, topo, q):
    try:
        os.environ.update(MV2AMD_CONTROL_PLANE_ONLY="1", MV2AMD_JOBID=jobid, RANK=str(rank), WORLD_SIZE=str(size),
                          LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(size))
        if topo is not None:
            os.environ["MV2AMD_TOPO"] = topo
        import mvapich2_amd as mm
        L = mm.lib()
        assert L.mv2h_init() == 0
        nl = ctypes.c_int()
        cols = (ctypes.c_int * (4 * size))()
        assert L.mv2h_get_topology(ctypes.byref(nl), cols, size) == 0
        got = [[cols[lv * size + r] for r in range(size)] for lv in range(nl.value)]
        assert L.mv2h_finalize() == 0
        q.put((rank, got))
    except BaseException as e:
        q.put((rank, repr(e)))


@pytest.mark.parametrize("topo,want", [("0,1,0,1", [[0, 1, 0, 1]]), ("0,0,1,1;0,1,0,1", [[0, 0, 1, 1], [0, 1, 0, 1]]),
                                       (None, None)])
def test_init_publishes_every_ranks_levels(topo, want):
    """MPI_Init: each rank derives its own ids (sysfs + CPU binding, or MV2AMD_TOPO) and every rank
    ends with the whole node's table; unbound ranks of one box agree on one table"""
    size = 4
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    jobid = "t" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_boot_worker, args=(r, size, jobid, topo, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    tables = list(res.values())
    assert all(isinstance(v, list) for v in tables), res
    assert all(v == tables[0] for v in tables), res
    if want is not None:
        assert tables[0] == want, tables[0]
    else:  # this container's processes share one binding: every level has one id for all ranks
        assert all(len(set(lv)) == 1 for lv in tables[0]), tables[0]
