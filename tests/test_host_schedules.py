"""CPU: the message schedules the host evaluates for a user op above 8 ranks (mpi/user_coll.cpp
BigEval, through the mv2h_host_sched_eval hook) against tests/ref_user.py's rank-by-rank
restatements, with a function that is neither commutative nor associative (inout = 2 in + 3 inout)
so that every operand order and bracketing shows.  ref_user's pt2pt_rs form (redscat_gather with
the allreduce pre-step) is itself pinned against the oracle's step-by-step pt2pt_rs."""
import ctypes

import numpy as np
import pytest

import mvapich2_amd as m
from mvapich2_amd.consts import OPS, TYPES
from oracle import oracle
from tests import ref_user

RD, PT2PT_RS, BINOMIAL, KNOMIAL, REDSCAT, RS_HALVING, RS_PAIRWISE, RS_RING, RING_CHUNK, RS_NONCOMM = range(10)
NS = [1, 2, 3, 5, 8, 9, 12, 13, 16, 17]


def fn(a, b):
    return (a.astype(np.int64) * 2 + b.astype(np.int64) * 3).astype(np.int32)


def operands(n, count, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(-50, 50, count).astype(np.int32) for _ in range(n)]


def hook(form, xs, me=0, root=0, k=2, commute=True):
    n, count = len(xs), len(xs[0])
    ops = np.ascontiguousarray(np.stack(xs))
    out = np.zeros(count, np.int32)
    rc = m.lib().mv2h_host_sched_eval(form, n, me, root, k, count, int(commute),
                                      ops.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return out


@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("commute", [True, False])
def test_recursive_doubling(n, commute):
    xs = operands(n, 7, n)
    want = ref_user.rd(xs, fn, commute)
    for me in range(n):
        assert np.array_equal(hook(RD, xs, me=me, commute=commute), want[me]), (n, me)


@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("count", [17, 40])
def test_pt2pt_rs_and_redscat_gather(n, count):
    xs = operands(n, count, 3 * n + count)
    if count >= ref_user.pof2_of(n):
        assert np.array_equal(hook(PT2PT_RS, xs), ref_user.redscat_gather(xs, fn, count, allreduce_pre=True)), n
        assert np.array_equal(hook(REDSCAT, xs), ref_user.redscat_gather(xs, fn, count)), n


@pytest.mark.parametrize("n", NS)
def test_binomial_and_knomial(n):
    xs = operands(n, 5, 11 * n)
    for root in sorted({0, n // 2, n - 1}):
        for commute in (True, False):
            assert np.array_equal(hook(BINOMIAL, xs, root=root, commute=commute),
                                  ref_user.binomial(xs, fn, root, commute)), (n, root, commute)
        for k in (2, 3, 4, 8):
            assert np.array_equal(hook(KNOMIAL, xs, root=root, k=k), ref_user.knomial(xs, fn, root, k)), (n, root, k)


@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("algo,form", [("rs_rec_halving", RS_HALVING), ("rs_pairwise", RS_PAIRWISE),
                                       ("rs_ring", RS_RING)])
def test_reduce_scatter_block(n, algo, form):
    """rank me's block from the operands' block me alone (the host path fetches only those)"""
    c = 3
    xs = operands(n, c * n, 5 * n)
    want = ref_user.reduce_scatter(xs, fn, TYPES["MPI_INT"][0], [c] * n, algo=algo)
    for me in range(n):
        blocks = [x[me * c:(me + 1) * c].copy() for x in xs]
        assert np.array_equal(hook(form, blocks, me=me), want[me]), (algo, n, me)


@pytest.mark.parametrize("n", NS)
def test_noncomm_reduce_scatter_block(n):
    """the host tree walk (BigEval::expr) of the non-commutative reduce-scatter's expression"""
    c = 2
    xs = operands(n, c * n, 13 * n)
    want = ref_user.reduce_scatter_noncomm(xs, fn, [c] * n)
    for me in range(n):
        blocks = [x[me * c:(me + 1) * c].copy() for x in xs]
        assert np.array_equal(hook(RS_NONCOMM, blocks, me=me, commute=False), want[me]), (n, me)


@pytest.mark.parametrize("n", NS)
def test_ring_chunk(n):
    cc = 4
    xs = operands(n, cc * n, 9 * n)
    want = ref_user.ring_chunks(xs, fn, cc * n)
    for me in range(n):
        chunk = [x[me * cc:(me + 1) * cc].copy() for x in xs]
        assert np.array_equal(hook(RING_CHUNK, chunk, me=me), want[me * cc:(me + 1) * cc]), (n, me)


@pytest.mark.parametrize("n", [3, 5, 9, 12, 13])
def test_ref_user_pt2pt_rs_matches_the_oracle(n):
    """ref_user's pt2pt_rs form against the oracle's pt2pt_rs with MPI_MAX on signed zeros / NaN
    payloads (where the operand order shows in the bits)"""
    H, OP, count = TYPES["MPI_DOUBLE"][0], OPS["MPI_MAX"], 37
    rng = np.random.default_rng(n)
    vals = np.array([0.0, -0.0, 1.0, -1.0, np.nan, -np.nan])
    xs = [rng.choice(vals, count).astype(np.float64) for _ in range(n)]

    def fmax(a, b):
        out = b.copy().view(np.uint8)
        assert oracle.reduce_local(a.copy().view(np.uint8), out, len(a), H, OP) == 0
        return out.view(np.float64)
    want = oracle.allreduce([x.view(np.uint8).copy() for x in xs], count, H, OP, algo=oracle.ALGOS.index("pt2pt_rs"))
    got = ref_user.redscat_gather(xs, fmax, count, allreduce_pre=True)
    assert np.array_equal(got.view(np.uint8), want[0])


def test_hook_rejects_bad_arguments():
    out = np.zeros(1, np.int32)
    ops = np.zeros(2, np.int32)
    L = m.lib()
    p = ops.ctypes.data_as(ctypes.c_void_p)
    q = out.ctypes.data_as(ctypes.c_void_p)
    assert L.mv2h_host_sched_eval(99, 2, 0, 0, 2, 1, 1, p, q) != 0
    assert L.mv2h_host_sched_eval(RD, 2, 2, 0, 2, 1, 1, p, q) != 0
    assert L.mv2h_host_sched_eval(RD, 0, 0, 0, 2, 1, 1, p, q) != 0
