"""n-input device reduction in the reference's orders vs the oracle's
simulation of the MV2 algorithms (bit-exact, fp included):
  LINEAR                  == two-level reduce_shmem  (oracle algo 1)
  BUTTERFLY, RS owners    == pt2pt_rs reduce-scatter (oracle algo 2)
  BUTTERFLY, fixed owner  == pt2pt_rd per rank        (oracle algo 3)"""
import ctypes

import numpy as np
import pytest

import mvapich2_amd as m
from mvapich2_amd.consts import DEVICE_UNSUPPORTED, OPS, TYPES, legal_pairs
from oracle import oracle
from tests.helpers import assert_bytes_equal, rand_typed

pytestmark = pytest.mark.gpu


def newrank_owner(r, n):
    pof2 = 1
    while pof2 * 2 <= n:
        pof2 *= 2
    rem = n - pof2
    if r < 2 * rem and r % 2 == 0:
        r += 1
    return r // 2 if r < 2 * rem else r - rem


def reduce_n(srcs, tname, op, count, order, owner):
    bufs = [m.DeviceBuffer.from_array(s) for s in srcs]
    ext = TYPES[tname][3]
    dst = m.DeviceBuffer(count * ext)
    arr = (ctypes.c_void_p * len(bufs))(*[b.ptr for b in bufs])
    rc = m.lib().mv2h_reduce_n(arr, len(bufs), dst.ptr, count, TYPES[tname][0], OPS[op], order, owner, None)
    assert rc == 0, rc
    return dst.download(np.uint8, count=count * ext)


SEL = [("MPI_SUM", "MPI_FLOAT"), ("MPI_SUM", "MPI_DOUBLE"), ("MPI_MAX", "MPI_FLOAT"), ("MPI_MIN", "MPI_DOUBLE"),
       ("MPI_PROD", "MPI_FLOAT"), ("MPI_SUM", "MPI_INT"), ("MPI_BXOR", "MPI_UNSIGNED_LONG"),
       ("MPI_LXOR", "MPI_FLOAT"), ("MPI_MAXLOC", "MPI_DOUBLE_INT"), ("MPI_MINLOC", "MPI_FLOAT_INT"),
       ("MPI_MAXLOC", "MPI_2REAL"), ("MPI_PROD", "MPI_C_FLOAT_COMPLEX"), ("MPI_SUM", "MPI_C_DOUBLE_COMPLEX"),
       ("MPI_MAX", "MPI_SHORT"), ("MPI_PROD", "MPI_SIGNED_CHAR")]


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 7, 8])
def test_orders_bit_exact(n):
    rng = np.random.default_rng(100 + n)
    for op, t in SEL:
        for count in (5, 1023):
            srcs = [rand_typed(t, count, rng, small=op == "MPI_PROD") for _ in range(n)]
            h, oh = TYPES[t][0], OPS[op]
            want = oracle.allreduce([s.copy() for s in srcs], count, h, oh, 1)[0]
            assert_bytes_equal(reduce_n(srcs, t, op, count, 0, 0), want, t, count, f"linear n={n} {op}")
            pof2 = 1
            while pof2 * 2 <= n:
                pof2 *= 2
            if count >= pof2:
                want = oracle.allreduce([s.copy() for s in srcs], count, h, oh, 2)[0]
                assert_bytes_equal(reduce_n(srcs, t, op, count, 1, -1), want, t, count, f"rs n={n} {op}")
            outs = oracle.allreduce([s.copy() for s in srcs], count, h, oh, 3)
            for r in range(n):
                got = reduce_n(srcs, t, op, count, 1, newrank_owner(r, n))
                assert_bytes_equal(got, outs[r], t, count, f"rd n={n} rank {r} {op}")


def test_golden_allred_cases_through_device_tree(golden):
    """allred.c / op*.c known answers reduced by the device tree in the order the
    reference's selection picks for that message size."""
    cases, arrs = golden
    for c in cases:
        if c["family"] not in ("allred", "op3") or c["type"] in DEVICE_UNSUPPORTED:
            continue
        n, count = c["n"], c["count"]
        ins = arrs[c["id"] + "__in"]
        sol = arrs[c["id"] + "__sol"]
        size = TYPES[c["type"]][2]
        srcs = [ins[r] for r in range(n)]
        if count * size <= 1024:
            got = reduce_n(srcs, c["type"], c["op"], count, 0, 0)
        else:
            got = reduce_n(srcs, c["type"], c["op"], count, 1, -1)
        assert_bytes_equal(got, sol, c["type"], count, c["id"])


def reduce_n_prog(srcs, tname, op, count, ps):
    bufs = [m.DeviceBuffer.from_array(s) for s in srcs]
    ext = TYPES[tname][3]
    dst = m.DeviceBuffer(count * ext)
    arr = (ctypes.c_void_p * len(bufs))(*[b.ptr for b in bufs])
    rc = m.lib().mv2h_reduce_n_prog(arr, len(bufs), dst.ptr, count, TYPES[tname][0], OPS[op], ctypes.byref(ps), None)
    assert rc == 0, rc
    return dst.download(np.uint8, count=count * ext)


def progset(coll, n, h, **kw):
    """the planner's raw program set (mv2h_plan) for one call"""
    L = m.lib()
    a, inner, unp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    ps = m.ProgSet()
    counts = kw.pop("counts", None)
    cz = (ctypes.c_size_t * n)(*counts) if counts else None
    m.check(L.mv2h_plan(m.COLL[coll], n, kw.get("rank", 0), kw.get("root", 0), kw.get("count", 0), cz, h, 0, 0,
                        ctypes.byref(a), ctypes.byref(inner), ctypes.byref(unp), ctypes.byref(ps)), "mv2h_plan")
    return a.value, ps


PROG_SEL = [("MPI_SUM", "MPI_FLOAT"), ("MPI_SUM", "MPI_DOUBLE"), ("MPI_MAX", "MPI_FLOAT"), ("MPI_MIN", "MPI_DOUBLE"),
            ("MPI_MAXLOC", "MPI_DOUBLE_INT"), ("MPI_PROD", "MPI_C_FLOAT_COMPLEX"), ("MPI_SUM", "MPI_C_DOUBLE_COMPLEX"),
            ("MPI_BXOR", "MPI_UNSIGNED_CHAR"), ("MPI_MINLOC", "MPI_SHORT_INT")]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 7, 8])
def test_program_evaluator_matches_oracle(n):
    """The device's program-order evaluator (prog_eval, kernels k_reduce_n / k_oneshot / k_pipe
    <.., PROG>) on the planner's programs: MPI_Reduce at every algorithm of the selection and
    root, the topology-aware allreduce tree, vs the oracle's rank-by-rank simulations."""
    rng = np.random.default_rng(500 + n)
    for op, t in PROG_SEL:
        h, oh = TYPES[t][0], OPS[op]
        size = TYPES[t][2]
        for nbytes in (400, 1600, 4096, 8192, 16384, 65536, 300000):
            count = max(1, nbytes // size)
            srcs = [rand_typed(t, count, rng, small=op == "MPI_PROD") for _ in range(n)]
            for root in sorted({0, n - 1}):
                algo, ps = progset("reduce", n, h, count=count, root=root)
                got = reduce_n_prog(srcs, t, op, count, ps)
                want = oracle.reduce_ref([s.view(np.uint8).ravel().copy() for s in srcs], count, h, oh, root)
                assert_bytes_equal(got, want, t, count, f"reduce n={n} {t} {op} count={count} root={root} "
                                                        f"algo={oracle.ALGOS[algo]}")
            if nbytes <= 2048:
                algo, ps = progset("allreduce", n, h, count=count)
                want = oracle.allreduce_ref([s.view(np.uint8).ravel().copy() for s in srcs], count, h, oh)[0]
                assert_bytes_equal(reduce_n_prog(srcs, t, op, count, ps), want, t, count,
                                   f"allreduce n={n} {t} {op} count={count} algo={oracle.ALGOS[algo]}")
