"""The N>1 decomposition of the device allreduce, on CPU.

Each rank owns the tiles t with t % n == rank and reduces them in the
reference's order (two-shot reduce-scatter), then every rank gathers the
owners' tiles (all-gather).  Two processes exchange data over torch.distributed
gloo exactly where the device kernel reads peers over xGMI; the assembled
result must equal the oracle's rank-by-rank simulation of MV2's
MPI_Allreduce bit for bit.  A single-process sweep covers n = 2..8."""
import os
import socket

import numpy as np
import pytest

from mvapich2_amd.consts import OPS, TYPES
from oracle import oracle
from tests import twoshot_model as tm
from tests.helpers import assert_bytes_equal, rand_typed

CASES = [("MPI_FLOAT", "MPI_SUM", 70001), ("MPI_DOUBLE", "MPI_MAX", 20011), ("MPI_INT", "MPI_PROD", 9000),
         ("MPI_DOUBLE_INT", "MPI_MAXLOC", 5003), ("MPI_FLOAT", "MPI_SUM", 100)]


def inputs(t, count, rank, seed):
    return rand_typed(t, count, np.random.default_rng(seed * 100 + rank), small=True).view(np.uint8).ravel().copy()


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
        for seed, (t, op, count) in enumerate(CASES):
            h, _, size, ext = TYPES[t]
            mine = inputs(t, count, rank, seed)
            # "remote reads" of the reduce-scatter phase
            allx = [torch.zeros(len(mine), dtype=torch.uint8) for _ in range(n)]
            dist.all_gather(allx, torch.from_numpy(mine))
            xs = [a.numpy() for a in allx]
            tp = tm.tree_params(n, count, size)
            tiles = tm.rs_tiles(xs, rank, count, ext, h, OPS[op], tp)
            # "remote reads" of the all-gather phase: owners' reduced tiles
            flat = np.zeros(count * ext, dtype=np.uint8)
            tv = tm.TV_BYTES
            for tt, data in tiles.items():
                flat[tt * tv:tt * tv + len(data)] = data
            allr = [torch.zeros(len(flat), dtype=torch.uint8) for _ in range(n)]
            dist.all_gather(allr, torch.from_numpy(flat))
            res = np.zeros(count * ext, dtype=np.uint8)
            nvec = count * ext // 16
            ntiles = (nvec + tv // 16 - 1) // (tv // 16)
            for tt in range(ntiles):
                own = allr[tt % n].numpy()
                res[tt * tv:min((tt + 1) * tv, nvec * 16)] = own[tt * tv:min((tt + 1) * tv, nvec * 16)]
            e0, tb = tm.tail(xs, count, ext, h, OPS[op], tp)
            res[e0 * ext:] = tb
            want = oracle.allreduce([x.copy() for x in xs], count, h, OPS[op])[rank]
            assert_bytes_equal(res, want, t, count, f"gloo rank {rank} {t} {op}")
        q.put((rank, "ok"))
    except BaseException as e:
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_twoshot_decomposition_gloo_world2():
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


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_twoshot_decomposition_single_process(n):
    for seed, (t, op, count) in enumerate(CASES):
        h, _, size, ext = TYPES[t]
        xs = [inputs(t, count, r, seed) for r in range(n)]
        tp = tm.tree_params(n, count, size)
        maps = [tm.rs_tiles(xs, r, count, ext, h, OPS[op], tp) for r in range(n)]
        res = tm.assemble(maps, count, ext, tm.tail(xs, count, ext, h, OPS[op], tp))
        want = oracle.allreduce([x.copy() for x in xs], count, h, OPS[op])
        for r in range(n):
            assert_bytes_equal(res, want[r], t, count, f"n={n} rank {r} {t} {op}")
