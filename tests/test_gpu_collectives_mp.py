"""Part (2) parity: the device collectives, one process per rank, several
ranks sharing the test box's single GPU (peers' arenas mapped through hipIpc
exactly as across GPUs).  Results are compared bit-exactly with the oracle's
simulation of the reference's algorithm for the same selection.  The "small"
geometry forces 3 workgroups x 4 KiB per round, so large cases run dozens of
rounds and reuse both arena parities within and across calls."""
import json
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

from mvapich2_amd.consts import DEVICE_UNSUPPORTED, OPS, TYPES
from oracle import oracle
from tests.helpers import as_bytes, assert_bytes_equal, rand_typed

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def inputs(case, rank):
    rng = np.random.default_rng(case["seed"] * 1000 + rank)
    return rand_typed(case["type"], case["count"], rng, small=case.get("small", False))


GEOMS = {"default": {}, "small": {"MV2AMD_PIPE_GRID": "3", "MV2AMD_PIPE_SUB": "4096"}}


def run_workers(n, cases, tmp_path, timeout=100, extra_env=None):
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"cases": cases}))
    out = tmp_path / "out"
    out.mkdir()
    jobid = "g" + uuid.uuid4().hex[:12]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MV2AMD_JOBID=jobid, MV2AMD_TIMEOUT_S="30", MV2AMD_DEVICE="0", **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_gpu_worker.py"), str(spec),
                                       str(out)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            logs.append(o.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-3000:]}"
    return lambda cid, r: np.load(out / f"{cid}_r{r}.npy")


def expected_allreduce(case, n):
    sends = [inputs(case, r) for r in range(n)]
    # IN_PLACE: the ring wrapper runs pt2pt_rs; MPI_Reduce keeps the pt2pt_rs order at every size
    algo = {"allreduce_inplace": 6, "reduce": 2}.get(case["kind"], -1)
    return oracle.allreduce([s.copy() for s in sends], case["count"], TYPES[case["type"]][0], OPS[case["op"]],
                            algo=algo)


BASIC = [("MPI_SUM", "MPI_FLOAT"), ("MPI_SUM", "MPI_DOUBLE"), ("MPI_MAX", "MPI_FLOAT"), ("MPI_MIN", "MPI_DOUBLE"),
         ("MPI_SUM", "MPI_INT"), ("MPI_PROD", "MPI_INT"), ("MPI_BXOR", "MPI_UNSIGNED_CHAR"), ("MPI_LAND", "MPI_C_BOOL"),
         ("MPI_MAXLOC", "MPI_DOUBLE_INT"), ("MPI_MINLOC", "MPI_2INT"), ("MPI_SUM", "MPI_C_FLOAT_COMPLEX"),
         ("MPI_MAXLOC", "MPI_SHORT_INT")]
COUNTS = [1, 3, 100, 4099, 70001, 300007]  # one-shot (<=256 KiB) and pipelined sizes, ragged tails


@pytest.mark.parametrize("n,geom", [(2, "default"), (3, "default"), (4, "default"), (3, "small"), (4, "small"),
                                    (7, "small"), (8, "default")])
def test_collectives_multiprocess(n, geom, tmp_path, golden):
    cases = []
    seed = 1
    for op, t in BASIC:
        for count in COUNTS:
            if t in ("MPI_SHORT_INT", "MPI_C_FLOAT_COMPLEX") and count > 5000:
                continue
            cases.append({"id": f"ar{seed}", "kind": "allreduce", "type": t, "op": op, "count": count,
                          "seed": seed, "small": op == "MPI_PROD"})
            seed += 1
    for op, t in (("MPI_SUM", "MPI_FLOAT"), ("MPI_MAXLOC", "MPI_DOUBLE_INT"), ("MPI_BXOR", "MPI_INT")):
        for count in (5, 70001):
            cases.append({"id": f"ia{seed}", "kind": "iallreduce", "type": t, "op": op, "count": count, "seed": seed})
            seed += 1
    for count in (10, 70001, 300007):
        cases.append({"id": f"ip{seed}", "kind": "allreduce_inplace", "type": "MPI_FLOAT", "op": "MPI_SUM",
                      "count": count, "seed": seed})
        seed += 1
    for count, root in ((5000, n - 1), (70001, 1), (300007, 0)):
        cases.append({"id": f"rd{seed}", "kind": "reduce", "type": "MPI_DOUBLE", "op": "MPI_SUM", "count": count,
                      "seed": seed, "root": root})
        seed += 1
    cases.append({"id": f"ar{seed}", "kind": "allreduce", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": 1 << 21,
                  "seed": seed})
    seed += 1
    # flat ring wrapper from 2 MiB (allreduce_osu.c:163-170): ragged remainders, chunks that are
    # not 16-byte multiples (padded staging), pair types, and IN_PLACE (pt2pt_rs on both ranges)
    for kind, t, op, count in (("allreduce", "MPI_FLOAT", "MPI_SUM", 524291), ("allreduce", "MPI_DOUBLE", "MPI_MAX", 262147),
                               ("allreduce", "MPI_DOUBLE_INT", "MPI_MAXLOC", 200003),
                               ("allreduce_inplace", "MPI_FLOAT", "MPI_SUM", 524291)):
        cases.append({"id": f"rg{seed}", "kind": kind, "type": t, "op": op, "count": count, "seed": seed})
        seed += 1
    for counts in ([1] * n, [1000 + r for r in range(n)], [70001] * n, [65536] * n, [0] + [33] * (n - 1)):
        cases.append({"id": f"rs{seed}", "kind": "reduce_scatter", "type": "MPI_INT", "op": "MPI_SUM",
                      "recvcounts": counts, "count": sum(counts), "seed": seed})
        seed += 1
    # floating point: ring order above 128 KiB total (red_scat_osu.c:1869-1880), linear below
    for t, op, counts in (("MPI_FLOAT", "MPI_SUM", [70001] * n), ("MPI_DOUBLE", "MPI_SUM", [20000 + r for r in range(n)]),
                          ("MPI_FLOAT", "MPI_MAX", [40000] * n), ("MPI_DOUBLE", "MPI_SUM", [100] * n),
                          ("MPI_DOUBLE_INT", "MPI_MINLOC", [9000] * n)):
        cases.append({"id": f"rs{seed}", "kind": "reduce_scatter", "type": t, "op": op,
                      "recvcounts": counts, "count": sum(counts), "seed": seed})
        seed += 1
    for count in (1, 13, 4096, 100003, 1 << 20):
        cases.append({"id": f"ag{seed}", "kind": "allgather", "type": "MPI_CHAR", "op": "MPI_SUM", "count": count,
                      "seed": seed})
        seed += 1
    for count in (1, 1000, 70001, 1 << 20):
        cases.append({"id": f"bc{seed}", "kind": "bcast", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": count,
                      "seed": seed, "root": 1 % n})
        seed += 1
    for commute in (0, 1):
        for count in (10, 1000, 524291):  # the last: ring wrapper for commutative ops (>= 2 MiB)
            cases.append({"id": f"uo{seed}", "kind": "user_allreduce", "count": count, "commute": commute,
                          "seed": seed, "type": "MPI_INT", "op": "MPI_SUM"})
            seed += 1
    for commute in (0, 1):
        for counts in ([10] * n, [50000 + r for r in range(n)]):
            cases.append({"id": f"ur{seed}", "kind": "user_reduce_scatter", "recvcounts": counts, "count": sum(counts),
                          "commute": commute, "seed": seed, "type": "MPI_INT", "op": "MPI_SUM"})
            seed += 1
    cases.append({"id": f"vb{seed}", "kind": "vector_bcast", "nblocks": 1000, "root": 0, "count": 8000,
                  "seed": seed, "type": "MPI_FLOAT", "op": "MPI_SUM"})
    seed += 1
    gcases, arrs = golden
    for c in gcases:
        if c["family"] == "allred" and c["n"] == n and c["type"] not in DEVICE_UNSUPPORTED:
            cases.append({"id": f"gd{seed}", "kind": "allreduce", "type": c["type"], "op": c["op"],
                          "count": c["count"], "seed": seed, "golden": c["id"]})
            seed += 1

    res = run_workers(n, cases, tmp_path, extra_env=GEOMS[geom])

    for case in cases:
        k, cid, t = case["kind"], case["id"], case.get("type")
        if k in ("allreduce", "allreduce_inplace") and "golden" in case:
            sol = arrs[case["golden"] + "__sol"]
            for r in range(n):
                assert_bytes_equal(res(cid, r), sol, t, case["count"], f"{cid} {case['golden']} rank {r}")
        elif k in ("allreduce", "allreduce_inplace", "iallreduce"):
            want = expected_allreduce(case, n)
            for r in range(n):
                assert_bytes_equal(res(cid, r), want[r], t, case["count"], f"{cid} {case['op']} n={n} rank {r}")
        elif k == "reduce":
            want = expected_allreduce(case, n)
            root = case["root"]
            assert_bytes_equal(res(cid, root), want[root], t, case["count"], f"{cid} reduce")
        elif k == "reduce_scatter":
            counts = case["recvcounts"]
            sends = [inputs(dict(case, count=sum(counts)), r) for r in range(n)]
            if sum(counts) * TYPES[t][2] >= 131072:
                full = oracle.reduce_scatter_ring(sends, counts, TYPES[t][0], OPS[case["op"]])
            else:
                full = oracle.reduce_linear(sends, sum(counts), TYPES[t][0], OPS[case["op"]])
            full = as_bytes(full)
            ext = TYPES[t][3]
            off = 0
            for r in range(n):
                assert_bytes_equal(res(cid, r), full[off * ext:(off + counts[r]) * ext], t, counts[r],
                                   f"{cid} {t} {case['op']} rank {r}")
                off += counts[r]
        elif k == "allgather":
            want = np.concatenate([as_bytes(inputs(case, r)) for r in range(n)])
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)
        elif k == "bcast":
            want = as_bytes(inputs(case, case["root"]))
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)
        elif k == "user_allreduce":
            want = user_allreduce_expected(n, case["count"], case["commute"])
            for r in range(n):
                assert np.array_equal(res(cid, r).view(np.int32), want[r]), (cid, r)
        elif k == "user_reduce_scatter":
            want = user_reduce_scatter_expected(n, case["recvcounts"], case["commute"])
            for r in range(n):
                assert np.array_equal(res(cid, r).view(np.int32), want[r]), (cid, r)
        elif k == "vector_bcast":
            nb = case["nblocks"]
            src = np.arange(nb * 8, dtype=np.float32).reshape(nb, 8)
            for r in range(n):
                got = res(cid, r).view(np.float32).reshape(nb, 8)
                assert np.array_equal(got[:, :4], src[:, :4]), (cid, r)
                if r != case["root"]:
                    assert np.all(got[:, 4:] == -1.0), "gap bytes of a vector type must not be written"


def user_allreduce_expected(n, count, commute):
    """Reference order for user ops (allreduce_osu.c): commutative & <= 1 KB ->
    two-level chain fn(x_i, acc); else recursive doubling with the
    dst < rank operand swap (:824-845) and the non-pof2 fold (:734-777)."""
    def fn(inp, io):
        return (inp * 2 + io * 3).astype(np.int32)
    xs = [((np.arange(count) + r) % 7).astype(np.int32) for r in range(n)]
    if commute and count * 4 <= 1024:
        acc = xs[0].copy()
        for i in range(1, n):
            acc = fn(xs[i], acc)
        return [acc] * n
    pof2 = 1
    while pof2 * 2 <= n:
        pof2 *= 2
    rem = n - pof2
    rb = [x.copy() for x in xs]
    newrank, real = [0] * n, [0] * pof2
    for r in range(n):
        if r < 2 * rem:
            if r % 2 == 0:
                newrank[r] = -1
            else:
                rb[r] = fn(xs[r - 1], rb[r])
                newrank[r] = r // 2
        else:
            newrank[r] = r - rem
        if newrank[r] >= 0:
            real[newrank[r]] = r
    mask = 1
    while mask < pof2:
        prev = [rb[real[nr]].copy() for nr in range(pof2)]
        for nr in range(pof2):
            r, dst = real[nr], real[nr ^ mask]
            tmp = prev[nr ^ mask]
            rb[r] = fn(tmp, rb[r]) if (commute or dst < r) else fn(rb[r], tmp)
        mask <<= 1
    for r in range(0, 2 * rem, 2):
        rb[r] = rb[r + 1]
    if commute and count * 4 >= (2 << 20) and count >= n:
        # ring wrapper (allreduce_osu.c:3758-3818): chunk c = fn chain from rank c along the
        # ring, received partial as inout; the remainder keeps the RD result above
        cc = count // n
        for c in range(n):
            blk = slice(c * cc, (c + 1) * cc)
            acc = xs[c][blk].copy()
            for k in range(1, n):
                acc = fn(xs[(c + k) % n][blk], acc)
            for r in range(n):
                rb[r] = rb[r].copy()
                rb[r][blk] = acc
    return rb


def user_reduce_scatter_expected(n, counts, commute):
    """User-op reduce-scatter orders (mpi_api.cpp user_reduce_scatter): commutative and
    >= 128 KiB total -> MPIR_Reduce_scatter_ring (red_scat_osu.c:1026-1180, own operand is
    inout at every hop); otherwise x_0 op x_1 op ... op x_{n-1} right to left."""
    def fn(inp, io):
        return (inp * 2 + io * 3).astype(np.int32)
    total = sum(counts)
    xs = [((np.arange(total) + r) % 7).astype(np.int32) for r in range(n)]
    out, off = [], 0
    for b in range(n):
        blk = slice(off, off + counts[b])
        if commute and total * 4 >= 131072:
            acc = xs[(b + 1) % n][blk]
            for k in range(2, n + 1):
                acc = fn(acc, xs[(b + k) % n][blk])
        else:
            acc = xs[n - 1][blk]
            for i in range(n - 2, -1, -1):
                acc = fn(xs[i][blk], acc)
        out.append(acc)
        off += counts[b]
    return out


KNOB_RUNS = [
    # MV2_ALLRED_USE_RING=0 (ch3_shmem_coll.c:2665-2670): >= 2 MiB stays in pt2pt_rs
    ({"MV2_ALLRED_USE_RING": "0"}, [("MPI_FLOAT", "MPI_SUM", 524291, 2)]),
    # MV2_ALLREDUCE_RING_ALGO_THRESHOLD (:3094-3098, K/M suffixes): the ring wrapper from 64 KiB
    ({"MV2_ALLREDUCE_RING_ALGO_THRESHOLD": "64K"}, [("MPI_FLOAT", "MPI_SUM", 70001, 4),
                                                    ("MPI_DOUBLE", "MPI_MAX", 10007, 4)]),
    # ring threshold 0: the small-message shortcut still wins up to 1 KiB (allreduce_osu.c:3155-3160),
    # everything above takes the ring wrapper (301 elements: padded chunks at n = 2, a remainder)
    ({"MV2_ALLREDUCE_RING_ALGO_THRESHOLD": "0"}, [("MPI_FLOAT", "MPI_SUM", 10, 1), ("MPI_FLOAT", "MPI_SUM", 301, 4)]),
    # MV2_COLL_SKIP_TABLE_THRESHOLD=0: no two-level shortcut, small calls take pt2pt_rs / RD
    ({"MV2_COLL_SKIP_TABLE_THRESHOLD": "0"}, [("MPI_FLOAT", "MPI_SUM", 10, 2), ("MPI_FLOAT", "MPI_SUM", 1, 2)]),
]


@pytest.mark.parametrize("n", [2, 3])
def test_mv2_selection_knobs(n, tmp_path):
    """The reference's MV2_* selection knobs move the algorithm (and so the reduction-order)
    boundaries; each run is checked bit-exactly against the oracle's algorithm for it."""
    seed = 900
    for i, (env, specs) in enumerate(KNOB_RUNS):
        cases = []
        for t, op, count, algo in specs:
            cases.append({"id": f"kn{seed}", "kind": "allreduce", "type": t, "op": op, "count": count,
                          "seed": seed, "algo": algo})
            seed += 1
        d = tmp_path / f"run{i}"
        d.mkdir()
        res = run_workers(n, cases, d, extra_env=env)
        for case in cases:
            sends = [inputs(case, r) for r in range(n)]
            want = oracle.allreduce([s.copy() for s in sends], case["count"], TYPES[case["type"]][0],
                                    OPS[case["op"]], algo=case["algo"])
            for r in range(n):
                assert_bytes_equal(res(case["id"], r), want[r], case["type"], case["count"],
                                   f"{case['id']} {env} rank {r}")
