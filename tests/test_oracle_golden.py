"""Pin the CPU oracle against the known answers of the reference's own test
suite (tests/golden, restated from test/mpi/coll/*.c by make_golden.py)."""
import numpy as np

from oracle import oracle
from tests.helpers import assert_bytes_equal


def _check_case(c, arrs):
    ins = arrs[c["id"] + "__in"]
    sol = arrs[c["id"] + "__sol"]
    n, count, th, oh, t = c["n"], c["count"], c["type_handle"], c["op_handle"], c["type"]
    fam = c["family"]
    if fam in ("allred", "op3"):
        outs = oracle.allreduce([ins[r].copy() for r in range(n)], count, th, oh)
        for r in range(n):
            assert_bytes_equal(outs[r], sol, t, count, f"{c['id']} rank {r} ({c['note']})")
    elif fam == "reduce_local":
        io = ins[1].copy()
        assert oracle.reduce_local(ins[0].copy(), io, count, th, oh) == 0
        assert_bytes_equal(io, sol, t, count, c["id"])
    elif fam == "redscat":
        full = oracle.reduce_linear([ins[r].copy() for r in range(n)], count, th, oh)
        assert np.array_equal(full.view(np.int32), sol.view(np.int32)), c["id"]
    else:
        raise AssertionError(fam)


def test_golden_manifest_covers_reference_tests(golden):
    cases, arrs = golden
    fams = {c["family"] for c in cases}
    assert fams == {"allred", "op3", "reduce_local", "redscat"}
    notes = {c["note"].split()[0] for c in cases}
    for src in ("allred.c", "opsum.c", "opprod.c", "opmax.c", "opmin.c", "opland.c", "oplor.c", "oplxor.c",
                "opband.c", "opbor.c", "opbxor.c", "opmaxloc.c", "opminloc.c", "reduce_local.c", "redscat.c"):
        assert src in notes, src
    assert len(cases) > 1000


def test_oracle_matches_every_golden_case(golden):
    cases, arrs = golden
    for c in cases:
        _check_case(c, arrs)


def test_oracle_algorithms_agree_on_exact_cases(golden):
    """two-level, recursive-halving and recursive-doubling give the known answer."""
    cases, arrs = golden
    for c in cases:
        if c["family"] != "allred" or c["count"] != 10:
            continue
        ins = arrs[c["id"] + "__in"]
        sol = arrs[c["id"] + "__sol"]
        for algo in (1, 2, 3):
            outs = oracle.allreduce([ins[r].copy() for r in range(c["n"])], c["count"], c["type_handle"],
                                    c["op_handle"], algo)
            for r in range(c["n"]):
                assert_bytes_equal(outs[r], sol, c["type"], c["count"], f"{c['id']} algo {algo}")


def test_round2_algorithms_reproduce_known_answers(golden):
    """Every restated algorithm of the one-node selection (topology-aware tree, binomial,
    knomial, redscat_gather, shmem reduce, reduce-scatter ring / recursive halving / pairwise /
    basic) reproduces the reference tests' known answers (allred.c, redscat.c)."""
    cases, arrs = golden
    seen = set()
    for c in cases:
        if c["family"] != "allred":
            continue
        ins = arrs[c["id"] + "__in"]
        sol = arrs[c["id"] + "__sol"]
        n, count, th, oh, t = c["n"], c["count"], c["type_handle"], c["op_handle"], c["type"]
        sends = [ins[r].copy() for r in range(n)]
        # the reference selection (topology-aware tree at these sizes), in place or not
        for ip in (False, True):
            outs = oracle.allreduce_ref([s.copy() for s in sends], count, th, oh, in_place=ip)
            for r in range(n):
                assert_bytes_equal(outs[r], sol, t, count, f"{c['id']} allreduce_ref rank {r}")
        # MPI_Reduce in every algorithm and at every root
        for algo in (1, 7, 8, 9, 14):
            if algo == 9 and count < 4:
                continue
            for root in range(n):
                out = oracle.reduce_ref([s.copy() for s in sends], count, th, oh, root, algo=algo)
                assert_bytes_equal(out, sol, t, count, f"{c['id']} reduce algo {algo} root {root}")
                seen.add(algo)
        # reduce-scatter of the same operands, equal blocks, every algorithm
        if count % n == 0 and c["op"] != "MPI_REPLACE":
            counts = [count // n] * n
            for algo in (10, 11, 12, 13):
                full = oracle.reduce_scatter_ref([s.copy() for s in sends], counts, th, oh, algo=algo)
                assert_bytes_equal(full, sol, t, count, f"{c['id']} reduce_scatter algo {algo}")
                seen.add(algo)
    assert seen >= {1, 7, 8, 9, 14, 10, 11, 12, 13}
    for c in cases:
        if c["family"] == "redscat":
            ins = arrs[c["id"] + "__in"]
            sol = arrs[c["id"] + "__sol"]
            n = c["n"]
            for algo in (-1, 10, 11, 12, 13):
                full = oracle.reduce_scatter_ref([ins[r].copy() for r in range(n)], [c["count"] // n] * n,
                                                 c["type_handle"], c["op_handle"], algo=algo)
                assert np.array_equal(full.view(np.int32), sol.view(np.int32)), (c["id"], algo)
