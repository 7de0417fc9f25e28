"""The N>1 decomposition of the device allreduce (k_pipe PIPE_AR), on CPU.

Each rank reduces its 16-byte-aligned segment in the reference's order from
the other ranks' arena slots and pushes the result to every peer's AG slot.
A host model of the segments, rounds, workgroup ranges and slots
(tests/pipe_model.py) must reproduce the oracle's rank-by-rank simulation of
MV2's MPI_Allreduce bit for bit, for n = 2..8 and geometries with several
rounds and workgroups.  A two-process gloo run exchanges the slot contents
over torch.distributed where the kernel stores into peers' arenas."""
import os
import socket

import numpy as np
import pytest

from mvapich2_amd.consts import OPS, TYPES
from oracle import oracle
from tests import pipe_model as pm
from tests.helpers import assert_bytes_equal, rand_typed

CASES = [("MPI_FLOAT", "MPI_SUM", 70001), ("MPI_DOUBLE", "MPI_MAX", 20011), ("MPI_INT", "MPI_PROD", 9000),
         ("MPI_DOUBLE_INT", "MPI_MAXLOC", 5003), ("MPI_FLOAT", "MPI_SUM", 100), ("MPI_SHORT_INT", "MPI_MINLOC", 3001),
         ("MPI_UNSIGNED_CHAR", "MPI_BXOR", 40003)]


def inputs(t, count, rank, seed):
    return rand_typed(t, count, np.random.default_rng(seed * 100 + rank), small=True).view(np.uint8).ravel().copy()


def test_geometry_matches_runtime_rules():
    # 256 MiB fp32 on 8 ranks: 32 MiB segments, 256 workgroups x 128 KiB, one round (default tiling)
    assert pm.pipe_geom(32 << 20) == (256, 128 << 10, 32 << 20, 1)
    # 256 MiB on 2 ranks: 128 MiB segments, 4 rounds; a tuned 128 x 256 KiB tiling keeps the slot size
    assert pm.pipe_geom(128 << 20) == (256, 128 << 10, 32 << 20, 4)
    assert pm.pipe_geom(128 << 20, pipe_grid=128, pipe_sub=256 << 10) == (128, 256 << 10, 32 << 20, 4)
    assert pm.pipe_geom(128 << 20, pipe_grid=256, pipe_sub=512 << 10)[1] == 128 << 10
    # 1 MiB segment: 64 workgroups x 16 KiB, one round
    assert pm.pipe_geom(1 << 20) == (64, 16 << 10, 1 << 20, 1)
    # tests sharing one GPU between 4 ranks: grid capped at cus / 4
    assert pm.pipe_geom(32 << 20, nshare=4)[0] == 64
    segs = pm.even_segments(1000003, 8)
    assert all(o % 16 == 0 for o, _ in segs) and sum(l for _, l in segs) == 1000003


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_pipe_allreduce_model_matches_oracle(n):
    for seed, (t, op, count) in enumerate(CASES):
        h, _, size, ext = TYPES[t]
        xs = [inputs(t, count, r, seed) for r in range(n)]
        tp = pm.tree_params(n, count, size)
        # small pipe_sub / grid: several rounds and workgroups per segment, ragged last ranges
        got = pm.allreduce(xs, count, ext, h, OPS[op], tp, geom_kw={"pipe_grid": 3, "pipe_sub": 4096})
        want = oracle.allreduce([x.copy() for x in xs], count, h, OPS[op])
        for r in range(n):
            assert_bytes_equal(got[r], want[r], t, count, f"n={n} rank {r} {t} {op}")


RING_CASES = [("MPI_FLOAT", "MPI_SUM", 4099), ("MPI_DOUBLE", "MPI_MAX", 2003), ("MPI_DOUBLE_INT", "MPI_MINLOC", 1001),
              ("MPI_FLOAT", "MPI_MIN", 3001)]


@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_ring_wrapper_model_matches_oracle(n):
    """MV2_ALLRED_USE_RING path (allreduce_osu.c:163-170, :3758-3818): ring over
    (count/n)*n elements as the pipe with ring segments, pt2pt_rs on the remainder."""
    for seed, (t, op, c0) in enumerate(RING_CASES):
        h, _, size, ext = TYPES[t]
        count = c0 * n + (n - 1)          # ragged: a remainder of n-1 elements
        xs = [inputs(t, count, r, seed + 50) for r in range(n)]
        main, rest = (count // n) * n, count - (count // n) * n
        tp = dict(pm.tree_params(n, main, size), ring_mode=True)
        got = pm.allreduce([x[:main * ext] for x in xs], main, ext, h, OPS[op], tp,
                           geom_kw={"pipe_grid": 3, "pipe_sub": 4096})
        # the remainder (< n elements) is a separate pt2pt_rs call (RD below pof2)
        tail = oracle.allreduce([x[main * ext:].copy() for x in xs], rest, h, OPS[op], algo=2)
        want = oracle.allreduce([x.copy() for x in xs], count, h, OPS[op], algo=4)
        for r in range(n):
            assert_bytes_equal(np.concatenate([got[r], tail[r]]), want[r], t, count, f"ring n={n} r{r} {t} {op}")


def test_ring_selection_thresholds():
    lib = oracle.lib()
    h = TYPES["MPI_FLOAT"][0]
    assert lib.oracle_allreduce_algo(8, 256, h) == 1          # 1024 B: skip-table two-level
    assert lib.oracle_allreduce_algo(8, 257, h) == 2
    assert lib.oracle_allreduce_algo(8, (2 << 20) // 4 - 1, h) == 2
    assert lib.oracle_allreduce_algo(8, (2 << 20) // 4, h) == 4   # ring wrapper from 2 MiB
    assert lib.oracle_allreduce_algo(8, 64 << 20, h) == 4          # the 256 MiB bench case


def test_ring_differs_from_butterfly_in_fp():
    """The selection matters for parity: at >= 2 MiB fp32 SUM the ring order and the
    pt2pt_rs butterfly give different bits for random operands."""
    n, count = 8, 1 << 19
    h = TYPES["MPI_FLOAT"][0]
    xs = [np.random.default_rng(r).standard_normal(count).astype(np.float32) for r in range(n)]
    ring = oracle.allreduce([x.copy() for x in xs], count, h, OPS["MPI_SUM"], algo=4)
    bfly = oracle.allreduce([x.copy() for x in xs], count, h, OPS["MPI_SUM"], algo=2)
    auto = oracle.allreduce([x.copy() for x in xs], count, h, OPS["MPI_SUM"])
    assert not np.array_equal(ring[0], bfly[0])
    assert np.array_equal(auto[0], ring[0])
    assert all(np.array_equal(ring[0], ring[r]) for r in range(n))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, n, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=n)
    try:
        for seed, (t, op, count) in enumerate(CASES[:4]):
            h, _, size, ext = TYPES[t]
            mine = inputs(t, count, rank, seed)
            nbytes = count * ext
            segs = pm.even_segments(nbytes, n)
            tp = pm.tree_params(n, count, size)
            # P1: my part of segment j goes to rank j (all_to_all of the segment slices)
            send = [torch.from_numpy(mine[o:o + ln].copy()) for o, ln in segs]
            myo, myl = segs[rank]
            recv = [torch.zeros(myl, dtype=torch.uint8) for _ in range(n)]
            reqs = []
            for j in range(n):
                if j == rank:
                    recv[j] = send[j]
                else:
                    reqs.append(dist.isend(send[j], j))
                    reqs.append(dist.irecv(recv[j], j))
            for r in reqs:
                r.wait()
            res = pm.reduce_range([r.numpy() for r in recv], myo // ext, ext, h, OPS[op], tp)
            # P2 push + P3 gather: every rank receives every reduced segment
            maxl = max(ln for _, ln in segs)
            pad = np.zeros(maxl, dtype=np.uint8)
            pad[:len(res)] = res
            allr = [torch.zeros(maxl, dtype=torch.uint8) for _ in range(n)]
            dist.all_gather(allr, torch.from_numpy(pad))
            out = np.zeros(nbytes, dtype=np.uint8)
            for j, (o, ln) in enumerate(segs):
                out[o:o + ln] = allr[j].numpy()[:ln]
            allx = [torch.zeros(len(mine), dtype=torch.uint8) for _ in range(n)]
            dist.all_gather(allx, torch.from_numpy(mine))
            xs = [a.numpy() for a in allx]
            want = oracle.allreduce([x.copy() for x in xs], count, h, OPS[op])[rank]
            assert_bytes_equal(out, want, t, count, f"gloo rank {rank} {t} {op}")
        q.put((rank, "ok"))
    except BaseException as e:
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_pipe_decomposition_gloo_world2():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


@pytest.mark.parametrize("n", [3, 8])
def test_ring_wrapper_in_place_is_two_rs_calls(n):
    """MPI_IN_PLACE at >= 2 MiB: the ring body rejects IN_PLACE (allreduce_osu.c:4095-4100), so
    the wrapper's result is pt2pt_rs over (count/n)*n elements followed by pt2pt_rs over the rest
    (for MAX/MIN the operand sides can differ from one whole-count call: ±0 ties, NaN payloads)."""
    count = (1 << 19) + n - 1
    h = TYPES["MPI_FLOAT"][0]
    xs = [np.random.default_rng(40 + r).standard_normal(count).astype(np.float32) for r in range(n)]
    main = (count // n) * n
    got = oracle.allreduce([x.copy() for x in xs], count, h, OPS["MPI_SUM"], algo=6)
    head = oracle.allreduce([x[:main].copy() for x in xs], main, h, OPS["MPI_SUM"], algo=2)
    tail = oracle.allreduce([x[main:].copy() for x in xs], count - main, h, OPS["MPI_SUM"], algo=2)
    whole = oracle.allreduce([x.copy() for x in xs], count, h, OPS["MPI_SUM"], algo=2)
    for r in range(n):
        assert np.array_equal(got[r], np.concatenate([head[r], tail[r]]))
    # for SUM the split changes only operand sides within the same pairing tree, and fp add is
    # commutative bit for bit, so the whole-count pt2pt_rs result agrees here
    for r in range(n):
        assert np.array_equal(got[r], whole[r])
