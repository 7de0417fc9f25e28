"""The product's algorithm selection and reduction-order programs
(runtime/orders.cpp, through the C-ABI mv2h_plan) against the oracle's
rank-by-rank simulation of the algorithms MVAPICH2 2.3.7 selects on one node.

The programs are evaluated on the host here (each step is one oracle
reduce_local call on the step's block), so a wrong tree is caught without a
GPU; the -m gpu tests then check the kernels that evaluate the same programs.
Inputs are fp with a wide dynamic range plus NaN payloads / signed zeros, so
any two different reduction orders give different bits.

Reference selections: MPIR_Allreduce_index_tuned_intra_MV2
(allreduce_osu.c:3015-3420), MPIR_Reduce_index_tuned_intra_MV2
(reduce_osu.c:2391-2660), MPIR_Reduce_scatter_MV2 (red_scat_osu.c:1771-1900)."""
import os

import numpy as np
import pytest

import mvapich2_amd as m
from mvapich2_amd.consts import OPS, TYPES
from oracle import oracle
from tests.helpers import assert_bytes_equal, rand_typed


def wide(t, count, rng):
    """fp operands whose sums depend on the association order"""
    x = rand_typed(t, count, rng)
    if TYPES[t][1] in ("f4", "f8"):
        scale = 10.0 ** rng.uniform(-4, 4, count)
        with np.errstate(all="ignore"):
            x = (x * scale).astype(x.dtype)
        if count > 12:
            x[:12] = rand_typed(t, 12, rng)  # NaN payloads, +-0, inf, denormals
    return x.view(np.uint8).ravel().copy()


def eval_progs(xs, progs, blk, e0, e1, ext, h, op):
    """Run per-block programs over elements [e0, e1) of the n operands (host)."""
    W = [x.copy() for x in xs]
    out = np.zeros((e1 - e0) * ext, dtype=np.uint8)
    e = e0
    while e < e1:
        b = 0 if len(progs) == 1 else min(e // blk, len(progs) - 1)
        be = e1 if b == len(progs) - 1 else min(e1, (b + 1) * blk)
        steps, res = progs[b]
        for d, s in steps:
            assert oracle.reduce_local(W[s][e * ext:be * ext], W[d][e * ext:be * ext], be - e, h, op) == 0
        out[(e - e0) * ext:(be - e0) * ext] = W[res][e * ext:be * ext]
        e = be
    return out


def allreduce_via_plan(xs, n, count, t, op, in_place=False):
    h, _, size, ext = TYPES[t]
    res = []
    for r in range(n):
        algo, _, _, progs, blk = m.plan("allreduce", n, r, h, count=count, in_place=in_place)
        if algo == 4:  # ring wrapper: ring over (count/n)*n unless IN_PLACE / count < n, pt2pt_rs on the rest
            main = 0 if (in_place or count < n) else (count // n) * n
            parts = []
            if main:
                parts.append(eval_progs(xs, progs, blk, 0, main, ext, h, OPS[op]))
            if main < count:
                a2, _, _, p2, b2 = m.plan("allreduce_rs", n, r, h, count=count - main, in_place=in_place)
                sub = [x[main * ext:] for x in xs]
                parts.append(eval_progs(sub, p2, b2, 0, count - main, ext, h, OPS[op]))
            res.append(np.concatenate(parts))
        else:
            res.append(eval_progs(xs, progs, blk, 0, count, ext, h, OPS[op]))
    return res


AR_COUNTS = [1, 3, 100, 256, 300, 512, 513, 700, 1000, 1024, 5000, 70001]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_allreduce_plan_matches_reference(n):
    rng = np.random.default_rng(1000 + n)
    for t, op in (("MPI_FLOAT", "MPI_SUM"), ("MPI_DOUBLE", "MPI_SUM"), ("MPI_FLOAT", "MPI_MAX")):
        h, _, size, ext = TYPES[t]
        for count in AR_COUNTS:
            xs = [wide(t, count, rng) for _ in range(n)]
            algo = m.plan("allreduce", n, 0, h, count=count)[0]
            assert algo == oracle.allreduce_select(n, count, h), (n, count, t)
            got = allreduce_via_plan(xs, n, count, t, op)
            want = oracle.allreduce_ref([x.copy() for x in xs], count, h, OPS[op])
            for r in range(n):
                assert_bytes_equal(got[r], want[r], t, count, f"allreduce n={n} count={count} {op} rank {r}")


def test_allreduce_default_selection_one_node():
    """Which algorithm each size takes on one node with the default knobs."""
    h = TYPES["MPI_FLOAT"][0]
    name = lambda n, c: oracle.ALGOS[m.plan("allreduce", n, 0, h, count=c)[0]]
    for n in range(3, 9):
        assert name(n, 1) == "topo_tree" and name(n, 512) == "topo_tree"   # 1 B .. 2 KiB
        assert name(n, 513) == "pt2pt_rs" and name(n, (2 << 20) // 4 - 1) == "pt2pt_rs"
        assert name(n, (2 << 20) // 4) == "ring_wrapper"
    # 2 ranks: the 2-ppn table keeps the two-level shmem path below 4 KiB
    assert name(2, 513) == "shmem_linear" and name(2, 1023) == "shmem_linear" and name(2, 1024) == "pt2pt_rs"


@pytest.mark.parametrize("n", [3, 8])
def test_allreduce_ring_and_in_place(n):
    rng = np.random.default_rng(77 + n)
    t, op = "MPI_FLOAT", "MPI_SUM"
    h = TYPES[t][0]
    for count in ((2 << 20) // 4 + 5, (2 << 20) // 4 * 2):
        xs = [wide(t, count, rng) for _ in range(n)]
        for ip in (False, True):
            got = allreduce_via_plan(xs, n, count, t, op, in_place=ip)
            want = oracle.allreduce_ref([x.copy() for x in xs], count, h, OPS[op], in_place=ip)
            for r in range(n):
                assert_bytes_equal(got[r], want[r], t, count, f"ring n={n} count={count} in_place={ip} rank {r}")


RED_COUNTS = [1, 2, 100, 256, 257, 600, 1024, 1500, 2048, 4096, 16384, 32768, 70001]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_reduce_plan_matches_reference(n):
    rng = np.random.default_rng(2000 + n)
    for t, op in (("MPI_FLOAT", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MIN"), ("MPI_DOUBLE_INT", "MPI_MAXLOC")):
        h, _, size, ext = TYPES[t]
        for count in RED_COUNTS:
            xs = [wide(t, count, rng) for _ in range(n)]
            for root in sorted({0, n - 1, n // 2}):
                algo, _, _, progs, blk = m.plan("reduce", n, root, h, count=count, root=root)
                assert algo == oracle.reduce_select(n, count, h)[0], (n, count, t)
                got = eval_progs(xs, progs, blk, 0, count, ext, h, OPS[op])
                want = oracle.reduce_ref([x.copy() for x in xs], count, h, OPS[op], root)
                assert_bytes_equal(got, want, t, count, f"reduce n={n} count={count} root={root} {op}")


def test_reduce_default_selection_one_node():
    """MPI_Reduce at 8 ranks with the CMA 16-ppn table (fp32 counts)."""
    h = TYPES["MPI_FLOAT"][0]
    name = lambda c: oracle.ALGOS[m.plan("reduce", 8, 0, h, count=c)[0]]
    assert name(256) == "shmem_linear"          # <= 1 KiB: shmem helper
    assert name(512) == "shmem_linear"          # 2 KiB: two-level table entry, stride <= 2048
    assert name(1024) == "knomial"              # 4 KiB
    assert name(2048) == "redscat_gather"       # 8 KiB
    assert name(4096) == "knomial"              # 16 KiB: two-level, stride > 2048
    assert name(16384) == "knomial"             # 64 KiB
    assert name(32768) == "redscat_gather"      # >= 128 KiB


RS_CASES = [(10, False), (64, False), (100, True), (1000, False), (1001, True), (4000, False), (9000, True),
            (20000, False), (40000, True)]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 7, 8])
def test_reduce_scatter_plan_matches_reference(n):
    rng = np.random.default_rng(3000 + n)
    for t, op in (("MPI_FLOAT", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MAX")):
        h, _, size, ext = TYPES[t]
        for per, ragged in RS_CASES:
            per = max(1, per // n)
            counts = [per + (rng.integers(0, 3) if ragged else 0) for _ in range(n)]
            total = sum(counts)
            xs = [wide(t, total, rng) for _ in range(n)]
            want = oracle.reduce_scatter_ref([x.copy() for x in xs], counts, h, OPS[op])
            assert m.plan("reduce_scatter", n, 0, h, counts=counts)[0] == oracle.reduce_scatter_select(counts, h)
            off = 0
            for r in range(n):
                algo, _, _, progs, blk = m.plan("reduce_scatter", n, r, h, counts=counts)
                got = eval_progs(xs, progs, blk, off, off + counts[r], ext, h, OPS[op])
                assert_bytes_equal(got, want[off * ext:(off + counts[r]) * ext], t, counts[r],
                                   f"reduce_scatter n={n} counts={counts} rank {r} algo {oracle.ALGOS[algo]}")
                off += counts[r]


KNOB_CASES = [
    ({"MV2_USE_TOPO_AWARE_ALLREDUCE": "0"}, {"use_topo_allreduce": 0}),
    ({"MV2_ENABLE_SKIP_TUNING_TABLE_SEARCH": "0"}, {"enable_skip_search": 0}),
    ({"MV2_ENABLE_TOPO_AWARE_COLLECTIVES": "0", "MV2_ENABLE_SKIP_TUNING_TABLE_SEARCH": "0"},
     {"enable_topo": 0, "enable_skip_search": 0}),
    ({"MV2_SHMEM_REDUCE_TREE_DEGREE": "2"}, {"tree_degree": 2}),
    ({"MV2_SMP_USE_CMA": "0"}, {"smp_use_cma": 0}),
    ({"MV2_USE_TOPO_AWARE_REDUCE": "1"}, {"use_topo_reduce": 1}),
    ({"MV2_USE_INTER_KNOMIAL_REDUCE_FACTOR": "2"}, {"inter_k": 2}),
    ({"MV2_ALLRED_USE_RING": "0", "MV2_RED_SCAT_RING_ALGO_THRESHOLD": "1K"},
     {"allred_use_ring": 0, "red_scat_ring_thr": 1024}),
    ({"MV2_COLL_SKIP_TABLE_THRESHOLD": "4096", "MV2_TOPO_AWARE_ALLREDUCE_MAX_MSG": "64"},
     {"coll_skip_thr": 4096, "topo_allred_max": 64}),
    # reduce_shmem from a lowered shmem slot on: MPICH's MPIR_Reduce_intra (binomial to 2 KiB,
    # redscat_gather above, allreduce_osu.c:1521-1526); the reduce helper's knomial from the slot
    ({"MV2_SHMEM_COLL_MAX_MSG_SIZE": "1024", "MV2_COLL_SKIP_TABLE_THRESHOLD": "8192",
      "MV2_TOPO_AWARE_ALLREDUCE_MAX_MSG": "64"},
     {"shmem_coll_max_msg": 1024, "coll_skip_thr": 8192, "topo_allred_max": 64}),
]


@pytest.mark.parametrize("env,kn", KNOB_CASES)
def test_knobs_move_selection_like_reference(env, kn, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    m.knobs_reload()
    try:
        knobs = oracle.default_knobs(**kn)
        rng = np.random.default_rng(5)
        t, op = "MPI_DOUBLE", "MPI_SUM"
        h, _, size, ext = TYPES[t]
        for n in (2, 5, 8):
            for count in (1, 40, 200, 300, 1100, 2048, 9000):
                xs = [wide(t, count, rng) for _ in range(n)]
                assert m.plan("allreduce", n, 0, h, count=count)[0] == oracle.allreduce_select(n, count, h, knobs=knobs)
                got = allreduce_via_plan(xs, n, count, t, op)
                want = oracle.allreduce_ref([x.copy() for x in xs], count, h, OPS[op], knobs=knobs)
                for r in range(n):
                    assert_bytes_equal(got[r], want[r], t, count, f"knobs {env} allreduce n={n} count={count} r{r}")
                root = n - 1
                algo, _, _, progs, blk = m.plan("reduce", n, root, h, count=count, root=root)
                assert algo == oracle.reduce_select(n, count, h, knobs=knobs)[0]
                got = eval_progs(xs, progs, blk, 0, count, ext, h, OPS[op])
                want = oracle.reduce_ref([x.copy() for x in xs], count, h, OPS[op], root, knobs=knobs)
                assert_bytes_equal(got, want, t, count, f"knobs {env} reduce n={n} count={count}")
                counts = [count // n + (1 if r < count % n else 0) for r in range(n)]
                if sum(counts):
                    want = oracle.reduce_scatter_ref([x.copy() for x in xs], counts, h, OPS[op], knobs=knobs)
                    off = 0
                    for r in range(n):
                        _, _, _, progs, blk = m.plan("reduce_scatter", n, r, h, counts=counts)
                        got = eval_progs(xs, progs, blk, off, off + counts[r], ext, h, OPS[op])
                        assert_bytes_equal(got, want[off * ext:(off + counts[r]) * ext], t, counts[r],
                                           f"knobs {env} reduce_scatter n={n} r{r}")
                        off += counts[r]
    finally:
        for k in env:
            monkeypatch.delenv(k, raising=False)
        m.knobs_reload()


def test_knomial_order_is_flagged_unpinned():
    """MPIR_Reduce_knomial_MV2 reduces in PMPI_Waitany completion order (reduce_osu.c:1766-1786):
    the reference's own fp result depends on arrival order, so the plan says so."""
    h = TYPES["MPI_FLOAT"][0]
    algo, _, unp, _, _ = m.plan("reduce", 8, 0, h, count=1024)
    assert oracle.ALGOS[algo] == "knomial" and unp == 1
    algo, _, unp, _, _ = m.plan("reduce", 8, 0, h, count=32768)
    assert oracle.ALGOS[algo] == "redscat_gather" and unp == 0


def test_user_op_kinds():
    """User ops: pt2pt_rs runs recursive doubling (allreduce_osu.c:802); non-commutative ops
    take recursive doubling everywhere and a binomial reduce rooted at 0 (reduce_osu.c:577-663)."""
    h = TYPES["MPI_FLOAT"][0]
    assert oracle.ALGOS[m.plan("allreduce", 8, 0, h, count=70001, opkind=1)[0]] == "pt2pt_rd"
    assert oracle.ALGOS[m.plan("allreduce", 8, 0, h, count=100, opkind=1)[0]] == "topo_tree"
    assert oracle.ALGOS[m.plan("allreduce", 8, 0, h, count=100, opkind=2)[0]] == "pt2pt_rd"
    assert oracle.ALGOS[m.plan("reduce", 8, 3, h, count=32768, root=3, opkind=1)[0]] == "binomial"
    assert oracle.ALGOS[m.plan("reduce", 8, 3, h, count=100, root=3, opkind=2)[0]] == "binomial"
    for n in (2, 3, 5, 8):
        for count in (5, 700, 5000):
            for opk in (1, 2):
                assert m.plan("allreduce", n, 0, h, count=count, opkind=opk)[0] == \
                    oracle.allreduce_select(n, count, h, opkind=opk)
                assert m.plan("reduce", n, 0, h, count=count, opkind=opk)[0] == \
                    oracle.reduce_select(n, count, h, opkind=opk)[0]


def eval_progs_fn(xs, progs, blk, e0, e1, fn):
    """host evaluation of plan programs with a user function fn(inp, io) -> io"""
    W = [x.copy() for x in xs]
    out = []
    e = e0
    while e < e1:
        b = 0 if len(progs) == 1 else min(e // blk, len(progs) - 1)
        be = e1 if b == len(progs) - 1 else min(e1, (b + 1) * blk)
        steps, res = progs[b]
        for d, s in steps:
            W[d][e:be] = fn(W[s][e:be], W[d][e:be])
        out.append(W[res][e:be].copy())
        e = be
    return np.concatenate(out) if out else xs[0][:0].copy()


@pytest.mark.parametrize("commute", [1, 0])
def test_user_op_plans_match_reference_restatement(commute):
    """The user-op host path evaluates these plans with the user function (mpi_api.cpp); here
    with the non-associative fn(in, io) = 2 in + 3 io against tests/ref_user.py."""
    from tests import ref_user
    fn = lambda a, b: (a * 2 + b * 3).astype(np.int32)
    h = TYPES["MPI_INT"][0]
    opk = 1 if commute else 2
    for n in (2, 3, 4, 6, 8):
        for count in (3, 100, 700, 5000, (2 << 20) // 4 + 3):
            xs = [((np.arange(count) * (r + 3)) % 11).astype(np.int32) for r in range(n)]
            want = ref_user.allreduce(xs, fn, commute, h, count)
            for r in range(n):
                algo, _, _, progs, blk = m.plan("allreduce", n, r, h, count=count, opkind=opk)
                if algo == 4:
                    main = (count // n) * n
                    _, _, _, p2, b2 = m.plan("allreduce_rs", n, r, h, count=count - main, opkind=opk)
                    got = np.concatenate([eval_progs_fn(xs, progs, blk, 0, main, fn),
                                          eval_progs_fn([x[main:] for x in xs], p2, b2, 0, count - main, fn)])
                else:
                    got = eval_progs_fn(xs, progs, blk, 0, count, fn)
                assert np.array_equal(got, want[r]), (n, count, r, oracle.ALGOS[algo])
            if count < 100000:
                for root in (0, n - 1):
                    _, _, _, progs, blk = m.plan("reduce", n, root, h, count=count, root=root, opkind=opk)
                    got = eval_progs_fn(xs, progs, blk, 0, count, fn)
                    assert np.array_equal(got, ref_user.reduce(xs, fn, commute, h, count, root)), (n, count, root)
            if commute:
                counts = [count // n + (1 if r < count % n else 0) for r in range(n)]
                want = ref_user.reduce_scatter(xs, fn, h, counts)
                off = 0
                for r in range(n):
                    _, _, _, progs, blk = m.plan("reduce_scatter", n, r, h, counts=counts, opkind=1)
                    got = eval_progs_fn(xs, progs, blk, off, off + counts[r], fn)
                    assert np.array_equal(got, want[r]), (n, counts, r)
                    off += counts[r]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_noncommutative_reduce_scatter_matches_reference(n):
    """MPIR_Reduce_scatter_non_comm_MV2 (red_scat_osu.c:1367-1760) for a non-commutative user op:
    the power-of-two / equal-count mirror-permuted halving (MPIR_Reduce_scatter_noncomm_MV2
    :132-290) and the recursive doubling with the non-power-of-two hand-off, against the rank-by-rank
    restatement tests/ref_user.reduce_scatter_noncomm, with the non-associative, non-commutative
    fn(in, io) = 2 in + 3 io."""
    from tests import ref_user
    fn = lambda a, b: (a * 2 + b * 3).astype(np.int64)
    h = TYPES["MPI_INT"][0]
    pof2 = 1 << (n - 1).bit_length()
    for counts in ([5] * n, [1] * n, [3 + (r % 3) for r in range(n)], [0] + [4] * (n - 1), [7] * (n - 1) + [2]):
        total = sum(counts)
        xs = [((np.arange(total) * (r + 3) + r) % 13).astype(np.int64) for r in range(n)]
        want = ref_user.reduce_scatter_noncomm(xs, fn, counts)
        regular = len(set(counts)) == 1
        # the blocking call, then MPI_Ireduce_scatter (ired_scat_osu.c:191-209) and, for equal
        # counts, the block forms (red_scat_block.c:614-640, ired_scat_block.c:910-920): one choice
        for kind in (None, "ireduce_scatter") + (("reduce_scatter_block",) if regular else ()):
            off = 0
            for r in range(n):
                if kind:
                    with m.nbc(kind):
                        algo, _, _, progs, blk = m.plan("reduce_scatter", n, r, h, counts=counts, opkind=2)
                else:
                    algo, _, _, progs, blk = m.plan("reduce_scatter", n, r, h, counts=counts, opkind=2)
                assert oracle.ALGOS[algo] == ("rs_noncomm_pof2" if pof2 == n and regular else "rs_noncomm_rd")
                got = eval_progs_fn(xs, progs, blk, off, off + counts[r], fn)
                assert np.array_equal(got, want[r]), (kind, n, counts, r, oracle.ALGOS[algo])
                off += counts[r]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 7, 8])
def test_nonblocking_plans_match_reference(n):
    """MPI_Iallreduce / MPI_Ireduce / MPI_Ireduce_scatter(_block) and the blocking
    MPI_Reduce_scatter_block take their own selections (oracle.iallreduce_select and
    friends, citing iallreduce_tuning.c / ireduce_tuning.c / ired_scat_tuning.c /
    red_scat_block.c); every rank of an Iallreduce gets rank 0's Ireduce result."""
    rng = np.random.default_rng(4000 + n)
    t, op = "MPI_FLOAT", "MPI_SUM"
    h, _, size, ext = TYPES[t]
    for count in (1, 3, 100, 512, 513, 1000, 5000, 70001):
        xs = [wide(t, count, rng) for _ in range(n)]
        with m.nbc("iallreduce"):
            want = oracle.iallreduce_ref([x.copy() for x in xs], count, h, OPS[op])
            for r in range(n):
                algo, _, _, progs, blk = m.plan("allreduce", n, r, h, count=count)
                assert algo == oracle.iallreduce_select(n, count, h)
                got = eval_progs(xs, progs, blk, 0, count, ext, h, OPS[op])
                assert_bytes_equal(got, want[r], t, count, f"iallreduce n={n} count={count} rank {r}")
        with m.nbc("ireduce"):
            root = n - 1
            algo, _, _, progs, blk = m.plan("reduce", n, root, h, count=count, root=root)
            assert oracle.ALGOS[algo] == "binomial"
            got = eval_progs(xs, progs, blk, 0, count, ext, h, OPS[op])
            want = oracle.ireduce_ref([x.copy() for x in xs], count, h, OPS[op], root)
            assert_bytes_equal(got, want, t, count, f"ireduce n={n} count={count}")
    for per in (1, 10, 1000, 40000):
        counts = [per] * n
        xs = [wide(t, per * n, rng) for _ in range(n)]
        for kind, algo_want in (("ireduce_scatter", oracle.ALGOS.index("rs_pairwise")),
                                ("reduce_scatter_block", oracle.reduce_scatter_block_select(n, per, h))):
            want = oracle.reduce_scatter_ref([x.copy() for x in xs], counts, h, OPS[op], algo=algo_want)
            with m.nbc(kind):
                for r in range(n):
                    algo, _, _, progs, blk = m.plan("reduce_scatter", n, r, h, counts=counts)
                    assert algo == algo_want, (kind, n, per)
                    got = eval_progs(xs, progs, blk, r * per, (r + 1) * per, ext, h, OPS[op])
                    assert_bytes_equal(got, want[r * per * ext:(r + 1) * per * ext], t, per, f"{kind} n={n} rank {r}")
    # outside the context the blocking selections come back
    assert oracle.ALGOS[m.plan("allreduce", n, 0, h, count=2)[0]] in ("topo_tree", "shmem_linear")
