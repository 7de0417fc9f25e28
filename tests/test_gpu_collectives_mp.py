"""Part (2) parity: the device collectives, one process per rank.  Each rank
takes GPU LOCAL_RANK % device_count, so on the 1-GPU test box all ranks share
one card (peers' arenas mapped through hipIpc exactly as across GPUs) and on
an 8-GPU node the same tests move every byte over xGMI.  Results are compared
bit-exactly with the oracle's rank-by-rank simulation of the algorithm
MVAPICH2 2.3.7 selects for the call (oracle.allreduce_ref / reduce_ref /
reduce_scatter_ref; user ops: tests/ref_user.py).  The "small" geometry
forces 3 workgroups x 4 KiB per round, so large cases run dozens of rounds and
reuse both arena parities within and across calls."""
import json
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

from mvapich2_amd.consts import DEVICE_UNSUPPORTED, OPS, TYPES
from oracle import oracle
from tests import ref_user
from tests.helpers import as_bytes, assert_bytes_equal, rand_typed

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def inputs(case, rank):
    rng = np.random.default_rng(case["seed"] * 1000 + rank)
    return rand_typed(case["type"], case["count"], rng, small=case.get("small", False),
                      ties=case.get("ties", False))


GEOMS = {"default": {}, "small": {"MV2AMD_PIPE_GRID": "3", "MV2AMD_PIPE_SUB": "4096"},
         # what a rank with a GPU to itself adopts, through the documented knobs:
         # full grids (the cap is max_grid / ranks per GPU), MPI_Init's tiling and one-shot crossover
         # probes with their 1 MiB one-shot slots, point-to-point copy kernels
         "full": {"MV2AMD_MAX_GRID": "8192", "MV2AMD_PIPE_AUTOTUNE": "1", "MV2AMD_P2P_KERNEL_COPY": "1"}}


def run_workers(n, cases, tmp_path, timeout=100, extra_env=None, ppn=None, expect_fail=False):
    """n ranks of tests/mp_gpu_worker.py; ppn < n emulates n / ppn nodes (node-major ranks,
    leaders linked over 127.0.0.1, runtime/internode.cpp).  expect_fail: return every rank's
    (exit code, log) instead of asserting success"""
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"cases": cases}))
    out = tmp_path / "out"
    out.mkdir()
    jobid = "g" + uuid.uuid4().hex[:12]
    ppn = ppn or n
    boot = {}
    if ppn < n:
        import socket
        so = socket.socket()
        so.bind(("127.0.0.1", 0))
        boot = {"MV2AMD_BOOT_ADDR": "127.0.0.1", "MV2AMD_BOOT_PORT": str(so.getsockname()[1]),
                "MV2AMD_NSHARE": str(n),  # every emulated node's ranks share the one GPU
                # the default 30 s: a device wait that runs out prints the epoch it waited for and
                # the flags it saw (coll.cpp check_err_word), so a stall names itself
                "MV2AMD_TIMEOUT_S": "30"}
        timeout = max(timeout, 240)
        so.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r % ppn), LOCAL_WORLD_SIZE=str(ppn),
                   MV2AMD_JOBID=jobid)
        env.update({"MV2AMD_TIMEOUT_S": "30", **boot, **(extra_env or {})})
        env.pop("MV2AMD_DEVICE", None)
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
    if expect_fail:
        return [(p.returncode, logs[r]) for r, p in enumerate(procs)]
    bad = [r for r, p in enumerate(procs) if p.returncode != 0]
    assert not bad, "ranks " + ", ".join(f"{r} (rc {procs[r].returncode})" for r in bad) + " failed:\n" + \
        "\n".join(f"--- rank {r}:\n{logs[r][-2000:]}" for r in range(n))
    return lambda cid, r: np.load(out / f"{cid}_r{r}.npy")


def expected_allreduce(case, n, knobs=None):
    """MPI_Allreduce as the reference runs it; MPI_Iallreduce: its own schedule (naive = Ireduce
    to rank 0 + Ibcast, iallreduce_tuning.c:184-190)"""
    sends = [inputs(case, r).view(np.uint8).ravel().copy() for r in range(n)]
    if case["kind"] == "iallreduce":
        return oracle.iallreduce_ref(sends, case["count"], TYPES[case["type"]][0], OPS[case["op"]])
    return oracle.allreduce_ref(sends, case["count"], TYPES[case["type"]][0], OPS[case["op"]],
                                in_place=case["kind"] == "allreduce_inplace", knobs=knobs)


def expected_reduce(case, n, knobs=None):
    sends = [inputs(case, r).view(np.uint8).ravel().copy() for r in range(n)]
    if case["kind"] == "ireduce":  # MPIR_Ireduce_binomial (ireduce_tuning.c default)
        return oracle.ireduce_ref(sends, case["count"], TYPES[case["type"]][0], OPS[case["op"]], case["root"])
    return oracle.reduce_ref(sends, case["count"], TYPES[case["type"]][0], OPS[case["op"]], case["root"],
                             knobs=knobs)


BASIC = [("MPI_SUM", "MPI_FLOAT"), ("MPI_SUM", "MPI_DOUBLE"), ("MPI_MAX", "MPI_FLOAT"), ("MPI_MIN", "MPI_DOUBLE"),
         ("MPI_SUM", "MPI_INT"), ("MPI_PROD", "MPI_INT"), ("MPI_BXOR", "MPI_UNSIGNED_CHAR"), ("MPI_LAND", "MPI_C_BOOL"),
         ("MPI_MAXLOC", "MPI_DOUBLE_INT"), ("MPI_MINLOC", "MPI_2INT"), ("MPI_SUM", "MPI_C_FLOAT_COMPLEX"),
         ("MPI_MAXLOC", "MPI_SHORT_INT")]
COUNTS = [1, 3, 100, 4099, 70001, 300007]  # one-shot (<=256 KiB) and pipelined sizes, ragged tails


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,geom", [(2, "default"), (3, "default"), (4, "default"), (3, "small"), (4, "small"),
                                    (7, "small"), (8, "default"), (2, "full"), (3, "full")])
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
    # nonblocking reduce and the block reduce-scatters: their own selections (fp, order-sensitive)
    for count, root in ((100, n - 1), (5000, 0), (300007, 1 % n)):
        cases.append({"id": f"ir{seed}", "kind": "ireduce", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": count,
                      "seed": seed, "root": root})
        seed += 1
    for via, per in (("block", 100), ("block", 70001), ("iblock", 1000), ("iblock", 140000), ("inb", 3000)):
        cases.append({"id": f"rb{seed}", "kind": "reduce_scatter", "type": "MPI_FLOAT", "op": "MPI_SUM", "via": via,
                      "recvcounts": [per] * n, "count": per * n, "seed": seed})
        seed += 1
    for count in (10, 70001, 300007):
        cases.append({"id": f"ip{seed}", "kind": "allreduce_inplace", "type": "MPI_FLOAT", "op": "MPI_SUM",
                      "count": count, "seed": seed})
        seed += 1
    # MPI_Reduce: shmem (<= 1 KiB and 2 KiB), knomial (4 KiB, 16 KiB, 64 KiB), redscat_gather
    # (8 KiB, >= 128 KiB), binomial (n = 2), at several roots; one-shot and pipelined sizes
    for t, op in (("MPI_FLOAT", "MPI_SUM"), ("MPI_DOUBLE", "MPI_SUM"), ("MPI_FLOAT", "MPI_MAX")):
        for count, root in ((100, n - 1), (512, 1 % n), (1024, 0), (2048, n - 1), (4096, 1 % n), (16384, 0),
                            (32768, n // 2), (300007, 1 % n)):
            if t == "MPI_DOUBLE":
                count //= 2
            cases.append({"id": f"rd{seed}", "kind": "reduce", "type": t, "op": op, "count": count,
                          "seed": seed, "root": root})
            seed += 1
    cases.append({"id": f"rd{seed}", "kind": "reduce", "type": "MPI_DOUBLE_INT", "op": "MPI_MAXLOC",
                  "count": 70001, "seed": seed, "root": n - 1})
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
    # x87 long double: reduced on the host in 80-bit (mpi_api.cpp ld_uop) in the reference's order
    for kind, op, count in (("allreduce", "MPI_SUM", 100), ("allreduce", "MPI_SUM", 70001),
                            ("allreduce", "MPI_MAX", 1000), ("reduce", "MPI_SUM", 30001)):
        cases.append({"id": f"x8{seed}", "kind": kind, "type": "MPI_LONG_DOUBLE", "op": op, "count": count,
                      "seed": seed, "root": n - 1})
        seed += 1
    cases.append({"id": f"x8{seed}", "kind": "reduce_scatter", "type": "MPI_LONG_DOUBLE", "op": "MPI_SUM",
                  "recvcounts": [5000 + r for r in range(n)], "count": sum(5000 + r for r in range(n)), "seed": seed})
    seed += 1
    # the same calls through the coll-function-table plugin (include/mv2amd_collops.h)
    for kind, t, op, count in (("allreduce", "MPI_FLOAT", "MPI_SUM", 301), ("allreduce", "MPI_DOUBLE", "MPI_SUM", 300007),
                               ("reduce", "MPI_FLOAT", "MPI_SUM", 70001)):
        cases.append({"id": f"co{seed}", "kind": kind, "type": t, "op": op, "count": count, "seed": seed,
                      "root": n - 1, "via": "collops"})
        seed += 1
    cases.append({"id": f"co{seed}", "kind": "reduce_scatter", "type": "MPI_FLOAT", "op": "MPI_SUM", "via": "collops",
                  "recvcounts": [9000 + r for r in range(n)], "count": sum(9000 + r for r in range(n)), "seed": seed})
    seed += 1
    cases.append({"id": f"co{seed}", "kind": "allgather", "type": "MPI_CHAR", "op": "MPI_SUM", "count": 100003,
                  "seed": seed, "via": "collops"})
    seed += 1
    cases.append({"id": f"co{seed}", "kind": "bcast", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": 70001,
                  "seed": seed, "root": 1 % n, "via": "collops"})
    seed += 1
    for counts in ([1] * n, [1000 + r for r in range(n)], [70001] * n, [65536] * n, [0] + [33] * (n - 1)):
        cases.append({"id": f"rs{seed}", "kind": "reduce_scatter", "type": "MPI_INT", "op": "MPI_SUM",
                      "recvcounts": counts, "count": sum(counts), "seed": seed})
        seed += 1
    # floating point in every reduce-scatter algorithm (red_scat_osu.c:1859-1896): basic (<= 256 B),
    # recursive halving (<= 16 KiB), pairwise (<= 64 KiB), ring (> 64 KiB)
    for t, op, counts in (("MPI_FLOAT", "MPI_SUM", [70001] * n), ("MPI_DOUBLE", "MPI_SUM", [20000 + r for r in range(n)]),
                          ("MPI_FLOAT", "MPI_MAX", [40000] * n), ("MPI_DOUBLE", "MPI_SUM", [100] * n),
                          ("MPI_DOUBLE_INT", "MPI_MINLOC", [9000] * n), ("MPI_FLOAT", "MPI_SUM", [4] * n),
                          ("MPI_FLOAT", "MPI_SUM", [3000 // n + r for r in range(n)]),
                          ("MPI_DOUBLE", "MPI_MAX", [6000 // n] * n), ("MPI_FLOAT", "MPI_SUM", [24000 // n] * n)):
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
        # the nonblocking and block forms (a non-commutative op: the same noncomm / rec_dbl choice)
        for via, counts in (("inb", [7 + (r % 3) for r in range(n)]), ("inb", [9] * n), ("block", [6] * n),
                            ("iblock", [6] * n), ("iblock", [3000] * n)):
            cases.append({"id": f"ur{seed}", "kind": "user_reduce_scatter", "recvcounts": counts, "count": sum(counts),
                          "commute": commute, "seed": seed, "type": "MPI_INT", "op": "MPI_SUM", "via": via})
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
        elif k in ("reduce", "ireduce"):
            want = expected_reduce(case, n)
            root = case["root"]
            assert_bytes_equal(res(cid, root), want, t, case["count"], f"{cid} reduce {t} {case['op']} "
                               f"count={case['count']} root={root}")
        elif k == "reduce_scatter":
            counts = case["recvcounts"]
            sends = [as_bytes(inputs(dict(case, count=sum(counts)), r)).copy() for r in range(n)]
            algo = -1
            if case.get("via") in ("block", "iblock"):  # MPICH reduce_scatter_block selection
                algo = oracle.reduce_scatter_block_select(n, counts[0], TYPES[t][0])
            elif case.get("via") == "inb":                # MPIR_Ireduce_scatter_pairwise
                algo = oracle.ALGOS.index("rs_pairwise")
            full = oracle.reduce_scatter_ref(sends, counts, TYPES[t][0], OPS[case["op"]], algo=algo)
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
            want = user_reduce_scatter_expected(n, case["recvcounts"], case["commute"], case.get("via"))
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


def ufn(inp, io):
    return (inp * 2 + io * 3).astype(np.int32)


def user_allreduce_expected(n, count, commute):
    """fn(in, io) = 2 in + 3 io in the order the reference takes for a user op (tests/ref_user.py)"""
    xs = [((np.arange(count) + r) % 7).astype(np.int32) for r in range(n)]
    return ref_user.allreduce(xs, ufn, commute, TYPES["MPI_INT"][0], count)


def user_reduce_scatter_expected(n, counts, commute, via=None):
    """commutative: MPIR_Reduce_scatter_MV2's choice (ref_user.reduce_scatter), MPI_Ireduce_scatter's
    pairwise, the block forms' MPICH selection; non-commutative: MPIR_Reduce_scatter_non_comm_MV2
    (ref_user.reduce_scatter_noncomm), which the nonblocking and block forms choose alike
    (ired_scat_osu.c:191-209, red_scat_block.c:614-640, ired_scat_block.c:910-920)"""
    total = sum(counts)
    xs = [((np.arange(total) + r) % 7).astype(np.int32) for r in range(n)]
    h = TYPES["MPI_INT"][0]
    if not commute:
        return ref_user.reduce_scatter_noncomm(xs, ufn, counts)
    if via == "inb":
        return ref_user.reduce_scatter(xs, ufn, h, counts, algo="rs_pairwise")
    if via in ("block", "iblock"):
        return ref_user.reduce_scatter(xs, ufn, h, counts, algo=oracle.ALGOS[oracle.reduce_scatter_block_select(n, counts[0], h)])
    return ref_user.reduce_scatter(xs, ufn, h, counts)


KNOB_RUNS = [
    # MV2_ALLRED_USE_RING=0 (ch3_shmem_coll.c:2665-2670): >= 2 MiB stays in pt2pt_rs
    ({"MV2_ALLRED_USE_RING": "0"}, {"allred_use_ring": 0}, [("MPI_FLOAT", "MPI_SUM", 524291)]),
    # MV2_ALLREDUCE_RING_ALGO_THRESHOLD (:3094-3098, K/M suffixes): the ring wrapper from 64 KiB
    ({"MV2_ALLREDUCE_RING_ALGO_THRESHOLD": "64K"}, {"ring_thr": 65536},
     [("MPI_FLOAT", "MPI_SUM", 70001), ("MPI_DOUBLE", "MPI_MAX", 10007)]),
    # ring threshold 0: the topology-aware tree still wins up to 2 KiB (allreduce_osu.c:120-133)
    ({"MV2_ALLREDUCE_RING_ALGO_THRESHOLD": "0"}, {"ring_thr": 0},
     [("MPI_FLOAT", "MPI_SUM", 10), ("MPI_FLOAT", "MPI_SUM", 301), ("MPI_FLOAT", "MPI_SUM", 601)]),
    # no topology-aware tree: two-level shmem up to 1 KiB, the tables above
    ({"MV2_USE_TOPO_AWARE_ALLREDUCE": "0"}, {"use_topo_allreduce": 0},
     [("MPI_FLOAT", "MPI_SUM", 10), ("MPI_DOUBLE", "MPI_SUM", 200), ("MPI_FLOAT", "MPI_SUM", 400)]),
    # tree degree 2 (MV2_SHMEM_REDUCE_TREE_DEGREE)
    ({"MV2_SHMEM_REDUCE_TREE_DEGREE": "2"}, {"tree_degree": 2}, [("MPI_FLOAT", "MPI_SUM", 77)]),
    # MV2_COLL_SKIP_TABLE_THRESHOLD=0 and no tree: small calls take the tables (pt2pt_rs / RD / two-level)
    ({"MV2_COLL_SKIP_TABLE_THRESHOLD": "0", "MV2_USE_TOPO_AWARE_ALLREDUCE": "0"},
     {"coll_skip_thr": 0, "use_topo_allreduce": 0}, [("MPI_FLOAT", "MPI_SUM", 10), ("MPI_FLOAT", "MPI_SUM", 1)]),
    # a lowered shmem slot (MV2_SHMEM_COLL_MAX_MSG_SIZE): reduce_shmem runs MPICH's MPIR_Reduce_intra
    # from it on (allreduce_osu.c:1521-1526: binomial to 2 KiB, redscat_gather above)
    ({"MV2_SHMEM_COLL_MAX_MSG_SIZE": "1024", "MV2_COLL_SKIP_TABLE_THRESHOLD": "8192",
      "MV2_TOPO_AWARE_ALLREDUCE_MAX_MSG": "64"},
     {"shmem_coll_max_msg": 1024, "coll_skip_thr": 8192, "topo_allred_max": 64},
     [("MPI_DOUBLE", "MPI_SUM", 200), ("MPI_DOUBLE", "MPI_SUM", 301), ("MPI_FLOAT", "MPI_MAX", 1500)]),
]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 3, 5])
def test_mv2_selection_knobs(n, tmp_path):
    """The reference's MV2_* selection knobs move the algorithm (and so the reduction-order)
    boundaries; each run is checked bit-exactly against the oracle with the same knobs."""
    seed = 900
    for i, (env, kn, specs) in enumerate(KNOB_RUNS):
        cases = []
        for t, op, count in specs:
            cases.append({"id": f"kn{seed}", "kind": "allreduce", "type": t, "op": op, "count": count, "seed": seed})
            seed += 1
            cases.append({"id": f"kr{seed}", "kind": "reduce", "type": t, "op": op, "count": count, "seed": seed,
                          "root": n - 1})
            seed += 1
        d = tmp_path / f"run{i}"
        d.mkdir()
        res = run_workers(n, cases, d, extra_env=env)
        knobs = oracle.default_knobs(**kn)
        for case in cases:
            if case["kind"] == "allreduce":
                want = expected_allreduce(case, n, knobs)
                for r in range(n):
                    assert_bytes_equal(res(case["id"], r), want[r], case["type"], case["count"],
                                       f"{case['id']} {env} rank {r}")
            else:
                want = expected_reduce(case, n, knobs)
                assert_bytes_equal(res(case["id"], n - 1), want, case["type"], case["count"], f"{case['id']} {env}")


@pytest.mark.timeout(400)
@pytest.mark.parametrize("n,xchg", [(2, None), (3, None), (8, None), (5, None), (3, "1")])
def test_user_op_on_strided_vector_operand(n, xchg, tmp_path):
    """configs[4]: MPI_Allreduce with a commutative user op on MPI_Type_vector(N, 4, 8, MPI_FLOAT)
    operands (the reference rejects predefined ops on derived types).  The result follows the
    reference's order for the call and only type-map bytes of recvbuf are written (gap bytes keep
    their -7.0): MPIR_Localcopy / uop calls touch the type map only.  The operands move packed
    and ring chunks are evaluated by their owner rank only (mpi/user_coll.cpp)."""
    cases = []
    sizes = [(64, 3), (1024, 40), (4096, 33), (262144, 5)]
    # 4096 x 16 B x 33 elements = 2.1 MiB: the ring wrapper with a remainder; 5 x 4 MiB: the ring
    # over 5 // n * n elements, recursive doubling on the rest (all of it at n = 8)
    if n == 8:
        sizes.append((4096, 1024))  # 64 MiB of payload (128 MiB span): the ring, one chunk per rank
    for seed, (nb, cnt) in enumerate(sizes, start=700):
        cases.append({"id": f"uv{seed}", "kind": "user_vector_allreduce", "nblocks": nb, "count": cnt,
                      "seed": seed})
    res = run_workers(n, cases, tmp_path, timeout=360, extra_env={"MV2AMD_UOP_EXCHANGE": xchg} if xchg else None)
    fn = lambda a, b: (a * np.float32(0.5) + b * np.float32(1.5)).astype(np.float32)
    for case in cases:
        nb, cnt = case["nblocks"], case["count"]
        ext_f = (nb - 1) * 8 + 4

        def typemap(x):  # (cnt, nb, 4) view of the type map
            return np.lib.stride_tricks.as_strided(x, (cnt, nb, 4), (ext_f * x.itemsize, 32, 4))

        def gaps(x):  # the 4 floats after each block but the last of every element
            return np.lib.stride_tricks.as_strided(x[4:], (cnt, nb - 1, 4), (ext_f * x.itemsize, 32, 4))
        packed = []
        for r in range(n):
            x = np.random.default_rng(case["seed"] * 1000 + r).standard_normal(cnt * ext_f).astype(np.float32)
            packed.append(typemap(x).reshape(cnt, nb * 4).copy())
            del x
        want = ref_user.allreduce(packed, fn, 1, None, cnt, nbytes=cnt * nb * 16)
        del packed
        for r in range(n):
            got = res(case["id"], r).view(np.float32)
            assert np.array_equal(typemap(got).reshape(cnt, nb * 4).view(np.uint32),
                                  want[r].reshape(cnt, nb * 4).view(np.uint32)), (case["id"], r)
            assert np.all(gaps(got) == -7.0), f"{case['id']} rank {r}: gap bytes of the vector type were written"
            # operands move reduce-scatter-shaped where the ring splits the work (count >= n): each
            # rank receives (n-1)/n of one packed operand (P) into a P-byte area; recursive doubling
            # (count < n) needs every operand whole
            inb, area = (int(v) for v in res(case["id"] + "_staged", r))
            P = cnt * nb * 16
            ring = cnt * nb * 16 >= (2 << 20) and cnt >= n  # the ring wrapper (2 MiB and up, n <= 8)
            algo = oracle.ALGOS[oracle.allreduce_select(n, P, 0x4c00010d, False, 1)]  # MPI_BYTE sizing
            if (algo == "pt2pt_rd" or (algo == "ring_wrapper" and cnt < n)) and (n >= 4 or xchg == "1"):
                # recursive doubling with its exchanges (user_coll.cpp run_rd_exchange, from 4
                # ranks on): one operand per step received, the pre- or post-step's included
                pof2 = ref_user.pof2_of(n)
                rem = n - pof2
                recvs = (1 if r < 2 * rem else 0) + (0 if (r < 2 * rem and r % 2 == 0) else pof2.bit_length() - 1)
                assert inb == recvs * P, (case["id"], r, inb, recvs, P)
            elif ring:
                chunk = cnt // n
                assert inb == (n - 1) * chunk * nb * 16 and area == n * chunk * nb * 16 <= P, \
                    (case["id"], r, inb, area, P)
            else:  # smaller: a tree order (split by ranges) or recursive doubling (whole operands)
                assert inb <= (n - 1) * P and (inb == (n - 1) * P or inb <= (n - 1) * -(-cnt // n) * nb * 16), \
                    (case["id"], r, inb, P)


@pytest.mark.timeout(480)
@pytest.mark.parametrize("n", [2, 4, 8])
def test_full_size_baseline_configs(n, tmp_path):
    """BASELINE configs[2]-[4] at their full sizes: 256 MiB fp32 SUM allreduce, 256 MiB
    reduce_scatter / allgather / bcast, 16 Mi-record MAXLOC on MPI_DOUBLE_INT; each rank checks
    its whole result against closed forms — and random N(0,1) fp32 allreduce / reduce_scatter at
    256 MiB bit-exact against the oracle's simulation of the reference's algorithm (ring wrapper
    and reduce-scatter ring)."""
    S = 256 << 20
    cases = [{"id": "bg1", "kind": "big_allreduce", "count": S // 4, "seed": 1},
             {"id": "bg2", "kind": "big_reduce_scatter", "count": S // 4, "seed": 2},
             {"id": "bg3", "kind": "big_allgather", "count": S // n, "seed": 3},
             {"id": "bg4", "kind": "big_bcast", "count": S, "seed": 4},
             {"id": "bg5", "kind": "big_maxloc", "count": S // 16, "seed": 5},
             {"id": "bg6", "kind": "big_allreduce_rand", "count": S // 4, "seed": 6},
             {"id": "bg7", "kind": "big_reduce_scatter_rand", "count": S // 4, "seed": 7}]
    res = run_workers(n, cases, tmp_path, timeout=400)
    for case in cases:
        for r in range(n):
            assert int(res(case["id"], r)[0]) == 0, (case["id"], r, int(res(case["id"], r)[0]))


@pytest.mark.timeout(400)
def test_allreduce_1gib_bit_exact(tmp_path):
    """configs[2]'s upper end: a 1 GiB fp32 SUM MPI_Allreduce of random N(0,1) operands at 2 ranks
    (the ring wrapper: 2 chunks of 512 MiB, each 16 rounds of the 32 MiB arena slots), every rank's
    whole result bit-exact against the oracle's simulation of the reference's ring."""
    n = 2
    cases = [{"id": "gb1", "kind": "big_allreduce_rand", "count": 1 << 28, "seed": 11}]
    res = run_workers(n, cases, tmp_path, timeout=360)
    for r in range(n):
        assert int(res("gb1", r)[0]) == 0, (r, int(res("gb1", r)[0]))


@pytest.mark.timeout(400)
@pytest.mark.parametrize("n", [4, 8])
def test_allreduce_1gib_n4_n8(n, tmp_path):
    """configs[2]'s 1 GiB point at 4 and 8 ranks (osu_allreduce.c:98-163 sweeps to -M): an exact
    integer-valued pattern checked over every element on every rank, then random N(0,1) operands
    whose result rank 0 checks bit-exactly against the oracle's ring on a 64 MiB slice (one slice
    inside each ring chunk; every rank regenerating 8 x 1 GiB of inputs would not fit the host)."""
    cases = [{"id": "gn1", "kind": "gib_allreduce", "count": 1 << 28, "slice": (16 << 20) // n, "seed": 13}]
    res = run_workers(n, cases, tmp_path, timeout=360)
    for r in range(n):
        assert [int(v) for v in res("gn1", r)] == [0, 0], (r, res("gn1", r))


@pytest.mark.timeout(600)
def test_operands_above_4gib(tmp_path):
    """MPI_Allreduce / MPI_Bcast / MPI_Reduce_local on 2^29 + 3 doubles (4 GiB + 24 B) at 2 ranks,
    MPI_Reduce_scatter / MPI_Allgather with 2 GiB + 8 B blocks: byte offsets past 32 bits in the
    pipelined kernels (ring chunks of 2 GiB + 8 B, the second starting off a 16-byte boundary), the
    one-element pt2pt_rs remainder and the streaming Reduce_local; exact closed-form results
    checked over every element in each rank."""
    n = 2
    cases = [{"id": "hg1", "kind": "huge", "count": (1 << 29) + 3, "seed": 1}]
    res = run_workers(n, cases, tmp_path, timeout=540)
    for r in range(n):
        assert [int(v) for v in res("hg1", r)] == [0] * 5, (r, res("hg1", r))


def test_mpit_counters_follow_the_selection(tmp_path):
    """MPI_T (mpi/mpit.cpp): a started counter handle counts the calls of the algorithms the
    reference's call chain runs for each call (its MPIR_T_PVAR_COUNTER_INC sites), 4 ranks:
      allreduce 8 B          topo-aware tree                     allreduce_osu.c:2279
      allreduce 4000 B       pt2pt_rs (16ppn table)              :640
      allreduce 524291 fp32  ring wrapper, ring body, pt2pt_rs on the 3-element remainder  :3762, :3899, :640
      allreduce 2 MiB IN_PLACE  ring wrapper, in-place body falls back to pt2pt_rs (:4095) :3762, :640
      reduce 400 B           two-level helper + MPIR_Reduce_shmem_MV2 (+ shmem coll call)  reduce_osu.c:2039, :1187
      reduce 4 KiB           knomial (CMA 16ppn table inter entry)                         :1672
      reduce_scatter 4x100 int   recursive halving                                         red_scat_osu.c:456
      reduce_scatter 4x70001 int ring                                                      :1039"""
    n = 4
    calls = [{"coll": "allreduce", "type": "MPI_FLOAT", "count": 2}, {"coll": "allreduce", "type": "MPI_FLOAT", "count": 1000},
             {"coll": "allreduce", "type": "MPI_FLOAT", "count": 524291},
             {"coll": "allreduce", "type": "MPI_FLOAT", "count": 524288, "in_place": True},
             {"coll": "reduce", "type": "MPI_FLOAT", "count": 100, "root": 1},
             {"coll": "reduce", "type": "MPI_FLOAT", "count": 1024, "root": 2},
             {"coll": "reduce_scatter", "type": "MPI_INT", "count": 100},
             {"coll": "reduce_scatter", "type": "MPI_INT", "count": 70001}]
    res = run_workers(n, [{"id": "mpit", "kind": "mpit_counts", "calls": calls}], tmp_path)
    want = {"mv2_coll_allreduce_topo_aware_hierarchical": 1, "mv2_coll_allreduce_shm_rs": 3,
            "mv2_coll_allreduce_pt2pt_ring_wrapper": 2, "mv2_coll_allreduce_pt2pt_ring": 1,
            "mv2_coll_reduce_two_level_helper": 1, "mv2_coll_reduce_shmem": 1, "mv2_num_shmem_coll_calls": 1,
            "mv2_coll_reduce_knomial": 1, "mv2_coll_reduce_scatter_rec_halving": 1, "mv2_coll_reduce_scatter_ring": 1}
    for r in range(n):
        got = json.loads(res("mpit", r).tobytes().decode())
        assert {k: v for k, v in got.items() if v} == want, (r, got)


@pytest.mark.parametrize("n", [2, 3])
def test_pipe_autotune_agrees_and_keeps_results(n, tmp_path):
    """MPI_Init's tiling autotune (coll.cpp pipe_autotune), forced on the shared GPU with a
    16 MiB probe: every rank adopts the same grid and bytes per workgroup (workgroup b of every
    rank pairs with workgroup b), and the calls after it stay bit-exact with the oracle (the
    tiling never changes the reduction order)."""
    cases = [{"id": "ti", "kind": "tiling_info"}]
    # sizes around the one-shot threshold the probe picks (16 KiB .. 1 MiB): the path never
    # changes a result
    for seed, (t, op, count) in enumerate((("MPI_FLOAT", "MPI_SUM", 1 << 21), ("MPI_DOUBLE", "MPI_SUM", 300007),
                                           ("MPI_FLOAT", "MPI_SUM", 70001), ("MPI_FLOAT", "MPI_SUM", 5000),
                                           ("MPI_FLOAT", "MPI_SUM", 12000), ("MPI_DOUBLE", "MPI_MAX", 20000),
                                           ("MPI_FLOAT", "MPI_SUM", 65536)), start=600):
        cases.append({"id": f"at{seed}", "kind": "allreduce", "type": t, "op": op, "count": count, "seed": seed})
    res = run_workers(n, cases, tmp_path, extra_env={"MV2AMD_PIPE_AUTOTUNE": "1",
                                                     "MV2AMD_PIPE_AUTOTUNE_BYTES": str(16 << 20)})
    infos = [res("ti", r).view(np.int64) for r in range(n)]
    assert infos[0][0] == 1 and infos[0][3] >= 1 and infos[0][6] >= 1, infos[0]
    assert (16 << 10) <= infos[0][5] <= (1 << 20), infos[0]  # the probe goes up to the 1 MiB slot
    assert infos[0][7] == 43, infos[0]  # MPI_Init's self-test: every cross-GPU kernel, graph lane included
    for r in range(1, n):
        assert np.array_equal(infos[r][:9], infos[0][:9]), (r, infos[r], infos[0])  # [9]: this rank's load time
    for case in cases[1:]:
        want = expected_allreduce(case, n)
        for r in range(n):
            assert_bytes_equal(res(case["id"], r), want[r], case["type"], case["count"], f"{case['id']} rank {r}")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,seed0", [(3, 5000), (4, 6000), (8, 7000)])
def test_random_sequence_of_collectives(n, seed0, tmp_path):
    """A seeded random sequence of 48 blocking and nonblocking collectives back to back — every
    kind, one-shot and pipelined sizes, ragged tails, several roots, types and ops — so that the
    arenas, epochs, completion words and plan cache are reused across kinds and sizes in orders no
    other test takes; every result bit-exact with the oracle."""
    rng = np.random.default_rng(seed0)
    kinds = ["allreduce", "allreduce_inplace", "iallreduce", "reduce", "ireduce", "reduce_scatter", "allgather",
             "bcast"]
    cases = []
    for i in range(48):
        k = kinds[int(rng.integers(len(kinds)))]
        op, t = BASIC[int(rng.integers(len(BASIC)))]
        if k in ("allgather", "bcast"):
            t, op = "MPI_CHAR" if k == "allgather" else "MPI_FLOAT", "MPI_SUM"
        count = int(rng.choice([1, 5, 777, 4099, 33333, 70001, 200003]))
        if t in ("MPI_SHORT_INT", "MPI_C_FLOAT_COMPLEX"):
            count = min(count, 4099)
        case = {"id": f"rq{seed0 + i}", "kind": k, "type": t, "op": op, "count": count, "seed": seed0 + i,
                "small": op == "MPI_PROD", "root": int(rng.integers(n))}
        if k == "reduce_scatter":
            counts = [count // n + int(rng.integers(0, 3)) for _ in range(n)]
            case.update(recvcounts=counts, count=sum(counts))
        cases.append(case)
    res = run_workers(n, cases, tmp_path)
    for case in cases:
        k, cid, t = case["kind"], case["id"], case["type"]
        if k in ("allreduce", "allreduce_inplace", "iallreduce"):
            want = expected_allreduce(case, n)
            for r in range(n):
                assert_bytes_equal(res(cid, r), want[r], t, case["count"], f"{cid} {k} {t} {case['op']} rank {r}")
        elif k in ("reduce", "ireduce"):
            want = expected_reduce(case, n)
            assert_bytes_equal(res(cid, case["root"]), want, t, case["count"], f"{cid} {k} {t} {case['op']}")
        elif k == "reduce_scatter":
            counts = case["recvcounts"]
            sends = [as_bytes(inputs(dict(case, count=sum(counts)), r)).copy() for r in range(n)]
            full = oracle.reduce_scatter_ref(sends, counts, TYPES[t][0], OPS[case["op"]])
            off, ext = 0, TYPES[t][3]
            for r in range(n):
                assert_bytes_equal(res(cid, r), full[off * ext:(off + counts[r]) * ext], t, counts[r], f"{cid} rank {r}")
                off += counts[r]
        elif k == "allgather":
            want = np.concatenate([as_bytes(inputs(case, r)) for r in range(n)])
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)
        else:
            want = as_bytes(inputs(case, case["root"]))
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)


def assert_refused_oversubscribed(out, n, tmp_path):
    """Every rank failed MPI_Init with the library's explicit refusal, and no result was written."""
    for r, (rc, log) in enumerate(out):
        assert rc != 0, f"rank {r} ran {n} processes on one GPU without an error:\n{log[-1500:]}"
        assert "processes share one GPU, more than the 8" in log, f"rank {r}: no refusal message:\n{log[-1500:]}"
        assert "MPI_Init" in log, log[-1500:]
    assert not list((tmp_path / "out").glob("*.npy")), "a rank wrote results"


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,ppn", [(9, 9), (12, 12), (10, 5)])
def test_more_than_8_processes_per_gpu_are_refused(n, ppn, tmp_path):
    """9 or 12 ranks of one node on the one GPU (nshare from the devices' PCI ids) and 10 = 2 x 5
    emulated nodes: MPI_Init refuses on every rank (MPI_ERR_UNSUPPORTED_OPERATION) instead of running
    collectives the GPU cannot keep exact (DESIGN.md "Ranks per GPU")."""
    case = {"id": "ar", "kind": "allreduce", "type": "MPI_INT", "op": "MPI_SUM", "count": 1000, "seed": 1}
    out = run_workers(n, [case], tmp_path, ppn=ppn, timeout=240, expect_fail=True)
    assert_refused_oversubscribed(out, n, tmp_path)


# (op, type) pairs whose result does not depend on the reduction order (wrapping integer arithmetic,
# bitwise and logical ops, integer MAX / MAXLOC): any algorithm's bits equal the one-node oracle's
ORDER_FREE = [("MPI_SUM", "MPI_INT"), ("MPI_PROD", "MPI_INT"), ("MPI_BXOR", "MPI_UNSIGNED_CHAR"),
              ("MPI_LAND", "MPI_C_BOOL"), ("MPI_MAX", "MPI_INT"), ("MPI_MAXLOC", "MPI_2INT"), ("MPI_BOR", "MPI_LONG")]


@pytest.mark.timeout(400)
@pytest.mark.parametrize("n,ppn,seed0,prog_max", [(6, 3, 8000, 8), (8, 4, 9000, 4), (12, 4, 9000, 8)])
def test_random_sequence_across_nodes(n, ppn, seed0, prog_max, tmp_path):
    """The random sequence on emulated nodes (node-major ranks, leaders over TCP; with prog_max 4 the
    8 ranks take the message schedules over the point-to-point channels that jobs above 8 ranks
    take), with order-free (op, type) pairs so that every multi-node algorithm must reproduce the
    one-node oracle's bits exactly.  Above 8 processes on the one GPU (12 = 3 x 4) MPI_Init must
    refuse the job on every rank with an explicit error, never return wrong bytes (DESIGN.md
    "Ranks per GPU": such jobs returned wrong sums in r05aa / r05ar / r06b)."""
    rng = np.random.default_rng(seed0)
    kinds = ["allreduce", "iallreduce", "reduce", "ireduce", "reduce_scatter", "allgather", "bcast"]
    cases = []
    for i in range(36):
        k = kinds[int(rng.integers(len(kinds)))]
        op, t = ORDER_FREE[int(rng.integers(len(ORDER_FREE)))]
        if k in ("allgather", "bcast"):
            t, op = "MPI_CHAR" if k == "allgather" else "MPI_INT", "MPI_SUM"
        count = int(rng.choice([1, 5, 777, 4099, 33333, 70001, 700003]))
        case = {"id": f"rn{seed0 + i}", "kind": k, "type": t, "op": op, "count": count, "seed": seed0 + i,
                "small": op == "MPI_PROD", "root": int(rng.integers(n))}
        if k == "reduce_scatter":
            counts = [count // n + int(rng.integers(0, 3)) for _ in range(n)]
            case.update(recvcounts=counts, count=sum(counts))
        cases.append(case)
    if n > 8:
        out = run_workers(n, cases, tmp_path, ppn=ppn, timeout=300, extra_env={"MV2AMD_MN_PROG_MAX": str(prog_max)},
                          expect_fail=True)
        assert_refused_oversubscribed(out, n, tmp_path)
        return
    res = run_workers(n, cases, tmp_path, ppn=ppn, timeout=300, extra_env={"MV2AMD_MN_PROG_MAX": str(prog_max)})
    for case in cases:
        k, cid, t = case["kind"], case["id"], case["type"]
        if k in ("allreduce", "iallreduce"):
            sends = [inputs(case, r).view(np.uint8).ravel().copy() for r in range(n)]
            want = oracle.allreduce_ref(sends, case["count"], TYPES[t][0], OPS[case["op"]])
            for r in range(n):
                assert_bytes_equal(res(cid, r), want[r], t, case["count"], f"{cid} {k} {t} {case['op']} rank {r}")
        elif k in ("reduce", "ireduce"):
            sends = [inputs(case, r).view(np.uint8).ravel().copy() for r in range(n)]
            want = oracle.reduce_ref(sends, case["count"], TYPES[t][0], OPS[case["op"]], case["root"])
            assert_bytes_equal(res(cid, case["root"]), want, t, case["count"], f"{cid} {k} {t} {case['op']}")
        elif k == "reduce_scatter":
            counts = case["recvcounts"]
            sends = [as_bytes(inputs(dict(case, count=sum(counts)), r)).copy() for r in range(n)]
            full = oracle.reduce_scatter_ref(sends, counts, TYPES[t][0], OPS[case["op"]])
            off, ext = 0, TYPES[t][3]
            for r in range(n):
                assert_bytes_equal(res(cid, r), full[off * ext:(off + counts[r]) * ext], t, counts[r], f"{cid} rank {r}")
                off += counts[r]
        elif k == "allgather":
            want = np.concatenate([as_bytes(inputs(case, r)) for r in range(n)])
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)
        else:
            want = as_bytes(inputs(case, case["root"]))
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)


PROTOCOL_VARIANTS = [
    # the full system-scope release MPI_Init's self-test falls back to when the light release fails
    # on a topology (coll.cpp coll_selftest) — never taken on a shared GPU by itself
    {"MV2AMD_LIGHT_RELEASE": "0"},
    # tilings the init-time autotune can adopt over xGMI (coll.cpp kGrid / kSub), with the
    # one-shot path narrowed so the pipelined kernel carries the small sizes too
    {"MV2AMD_PIPE_GRID": "64", "MV2AMD_PIPE_SUB": str(512 << 10)},
    {"MV2AMD_PIPE_GRID": "256", "MV2AMD_PIPE_SUB": str(16 << 10), "MV2AMD_ONESHOT_MAX": str(16 << 10)},
]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("vi", range(len(PROTOCOL_VARIANTS)))
def test_release_and_tiling_variants(n, vi, tmp_path):
    """The cross-process protocol under the settings a one-rank-per-GPU node may adopt at
    MPI_Init: the full-release fallback and non-default tilings.  Every collective stays
    bit-exact with the oracle (the tiling and the release never change a reduction order)."""
    env = PROTOCOL_VARIANTS[vi]
    cases, seed = [], 4000
    for t, op, count in (("MPI_FLOAT", "MPI_SUM", 1000), ("MPI_FLOAT", "MPI_SUM", 70001),
                         ("MPI_DOUBLE", "MPI_MAX", 300007), ("MPI_FLOAT", "MPI_SUM", (1 << 20) + 3),
                         ("MPI_FLOAT", "MPI_SUM", 524291), ("MPI_DOUBLE_INT", "MPI_MAXLOC", 70001)):
        cases.append({"id": f"pv{seed}", "kind": "allreduce", "type": t, "op": op, "count": count, "seed": seed})
        seed += 1
    for count, root in ((4096, 1 % n), (300007, n - 1)):
        cases.append({"id": f"pv{seed}", "kind": "reduce", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": count,
                      "seed": seed, "root": root})
        seed += 1
    for counts in ([70001] * n, [1000 + r for r in range(n)]):
        cases.append({"id": f"pv{seed}", "kind": "reduce_scatter", "type": "MPI_FLOAT", "op": "MPI_SUM",
                      "recvcounts": counts, "count": sum(counts), "seed": seed})
        seed += 1
    cases.append({"id": f"pv{seed}", "kind": "allgather", "type": "MPI_CHAR", "op": "MPI_SUM", "count": 1 << 20,
                  "seed": seed})
    seed += 1
    cases.append({"id": f"pv{seed}", "kind": "bcast", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": 300007,
                  "seed": seed, "root": n - 1})
    res = run_workers(n, cases, tmp_path, extra_env=env)
    for case in cases:
        k, cid, t = case["kind"], case["id"], case["type"]
        if k == "allreduce":
            want = expected_allreduce(case, n)
            for r in range(n):
                assert_bytes_equal(res(cid, r), want[r], t, case["count"], f"{cid} {env} rank {r}")
        elif k == "reduce":
            want = expected_reduce(case, n)
            assert_bytes_equal(res(cid, case["root"]), want, t, case["count"], f"{cid} {env}")
        elif k == "reduce_scatter":
            counts = case["recvcounts"]
            sends = [as_bytes(inputs(dict(case, count=sum(counts)), r)).copy() for r in range(n)]
            full = oracle.reduce_scatter_ref(sends, counts, TYPES[t][0], OPS[case["op"]])
            off, ext = 0, TYPES[t][3]
            for r in range(n):
                assert_bytes_equal(res(cid, r), full[off * ext:(off + counts[r]) * ext], t, counts[r],
                                   f"{cid} {env} rank {r}")
                off += counts[r]
        elif k == "allgather":
            want = np.concatenate([as_bytes(inputs(case, r)) for r in range(n)])
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)
        else:
            want = as_bytes(inputs(case, case["root"]))
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)


@pytest.mark.parametrize("n", [2, 3])
def test_stream_ordered_collectives(n, tmp_path):
    """MPIX_*_enqueue (mv2h.h stream-ordered collectives): a chain of calls on one HIP stream,
    the second reading the first's result in stream order, a blocking MPI_Allreduce between them
    (ordered after the queued calls), one host synchronisation at the end; every result is
    bit-exact with the oracle's simulation of the algorithm the blocking call would take."""
    cases = []
    for seed, c in ((501, 1000), (502, (1 << 20) + 5)):
        counts = [c // n + (1 if r < c % n else 0) for r in range(n)]
        cases.append({"id": f"eq{seed}", "kind": "enqueue_seq", "type": "MPI_FLOAT", "count": c, "seed": seed,
                      "recvcounts": counts, "per": c // n})
    res = run_workers(n, cases, tmp_path)
    F, SUM, MAX = TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"], OPS["MPI_MAX"]
    for case in cases:
        c, counts, per = case["count"], case["recvcounts"], case["per"]
        xs = [inputs(case, r).view(np.uint8).ravel().copy() for r in range(n)]
        y = oracle.allreduce_ref(xs, c, F, SUM)
        z = oracle.allreduce_ref([y[r].copy() for r in range(n)], c, F, SUM)
        rs_full = oracle.reduce_scatter_ref([x.copy() for x in xs], counts, F, SUM)
        ag = np.concatenate([x[:per * 4] for x in xs])
        red = oracle.reduce_ref([x.copy() for x in xs], c, F, MAX, 0)
        for r in range(n):
            got = res(case["id"], r)
            o = 0
            parts = {}
            for name, nb in (("y", c * 4), ("z", c * 4), ("xb", c * 4), ("w", c * 4), ("rs", counts[r] * 4),
                             ("ag", per * n * 4), ("r", c * 4), ("w2", c * 4)):
                parts[name] = got[o:o + nb]
                o += nb
            tag = f"{case['id']} rank {r}"
            assert_bytes_equal(parts["y"], y[r], "MPI_FLOAT", c, tag + " y")
            assert_bytes_equal(parts["z"], z[r], "MPI_FLOAT", c, tag + " z")
            assert np.array_equal(parts["xb"], xs[1 % n]), tag + " bcast"
            assert_bytes_equal(parts["w"], y[r], "MPI_FLOAT", c, tag + " blocking w")
            assert_bytes_equal(parts["w2"], y[r], "MPI_FLOAT", c, tag + " blocking w2 after hipStreamDestroy")
            off = sum(counts[:r]) * 4
            assert_bytes_equal(parts["rs"], rs_full[off:off + counts[r] * 4], "MPI_FLOAT", counts[r], tag + " rs")
            assert np.array_equal(parts["ag"], ag), tag + " allgather"
            if r == 0:
                assert_bytes_equal(parts["r"], red, "MPI_FLOAT", c, tag + " reduce")


@pytest.mark.parametrize("n", [2, 3])
def test_graph_captured_allreduce(n, tmp_path):
    """MPIX_Allreduce_enqueue captured into HIP graphs (the graph lane: own arenas, epochs and
    parities read from the device and advanced by the kernels), one graph per size (one-shot,
    pipelined ring with a remainder), each replayed three times with new operands and a blocking
    MPI_Allreduce in between; every replay bit-exact with the oracle."""
    counts, reps = [1000, (1 << 20) + 5], 3
    case = {"id": "gr", "kind": "graph_allreduce", "counts": counts, "reps": reps, "seed": 77}
    res = run_workers(n, [case], tmp_path)
    F, SUM = TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]
    got = [res("gr", r) for r in range(n)]
    off = 0
    for k in range(reps):
        for g, c in enumerate(counts):
            xs = [np.random.default_rng(77 * 100000 + k * 1000 + g * 10 + r).standard_normal(c).astype(np.float32)
                  .view(np.uint8) for r in range(n)]
            want = oracle.allreduce_ref(xs, c, F, SUM)
            for r in range(n):
                assert_bytes_equal(got[r][off:off + c * 4], want[r], "MPI_FLOAT", c, f"replay {k} count {c} rank {r}")
            off += c * 4
        xs = [np.random.default_rng(77 * 7 + k * 13 + r).standard_normal(4096).astype(np.float32).view(np.uint8)
              for r in range(n)]
        want = oracle.allreduce_ref(xs, 4096, F, SUM)
        for r in range(n):
            assert_bytes_equal(got[r][off:off + 4096 * 4], want[r], "MPI_FLOAT", 4096, f"host lane after replay {k} rank {r}")
        off += 4096 * 4


@pytest.mark.parametrize("n", [2, 3, 4])
def test_graph_captured_collectives(n, tmp_path):
    """Every stream-ordered collective captured into one HIP graph (reduce-scatter, allgather,
    broadcast, reduce, allreduce back to back; the one-shot kernels at 3 and 100 elements per
    rank — 3 is a byte-wise allgather block — the pipelined kernels at 300,007), each graph
    replayed four times with new operands and a blocking MPI_Allgather between replays; every
    result checked against its closed form (mp_gpu_worker.graph_collectives)."""
    case = {"id": "gc", "kind": "graph_collectives", "counts": [3, 100, 300007], "reps": 4}
    res = run_workers(n, [case], tmp_path)
    for r in range(n):
        assert res("gc", r)[0] == 0, f"rank {r}: {int(res('gc', r)[0])} wrong results"


@pytest.mark.parametrize("n,topo", [(4, "0,1,0,1"), (8, "0,1,0,1,0,1,0,1"), (8, "0,0,1,1,2,2,3,3;0,0,0,0,1,1,1,1")])
def test_gpu_topology_levels(n, topo, tmp_path):
    """The topology-aware shm tree over several levels (MV2AMD_TOPO sets every rank's NUMA / socket
    ids; MPI_Init publishes them): small allreduces (<= 2 KiB) and topology-aware reduces on the
    device, bit-exact with the oracle's multi-level simulation (tests/test_topology.py restates the
    levels on the CPU)."""
    levels = [[int(c) for c in lv.split(",")] for lv in topo.split(";")]
    cases = []
    for seed, (t, op, count) in enumerate((("MPI_FLOAT", "MPI_SUM", 7), ("MPI_DOUBLE", "MPI_SUM", 100),
                                           ("MPI_FLOAT", "MPI_MAX", 500), ("MPI_FLOAT", "MPI_SUM", 512)), start=950):
        cases.append({"id": f"tp{seed}", "kind": "allreduce", "type": t, "op": op, "count": count, "seed": seed})
        cases.append({"id": f"tr{seed}", "kind": "reduce", "type": t, "op": op, "count": count, "seed": seed,
                      "root": n - 1})
    res = run_workers(n, cases, tmp_path, extra_env={"MV2AMD_TOPO": topo, "MV2_USE_TOPO_AWARE_REDUCE": "1"})
    oracle.set_topology(levels, n)
    try:
        knobs = oracle.default_knobs(use_topo_reduce=1)
        for case in cases:
            if case["kind"] == "allreduce":
                want = expected_allreduce(case, n, knobs)
                for r in range(n):
                    assert_bytes_equal(res(case["id"], r), want[r], case["type"], case["count"], f"{case['id']} {topo} rank {r}")
            else:
                want = expected_reduce(case, n, knobs)
                assert_bytes_equal(res(case["id"], n - 1), want, case["type"], case["count"], f"{case['id']} {topo}")
    finally:
        oracle.set_topology([], n)


@pytest.mark.parametrize("n", [2, 3])
def test_derived_type_calls_make_no_device_allocations(n, tmp_path):
    """Derived-type MPI_Bcast / MPI_Allgather and non-contiguous MPI_Isend / MPI_Irecv stage
    through pooled device temporaries (runtime/world.cpp pool_get): after one warm-up round, ten
    more rounds make no hipMalloc inside the calls (mv2h_get_info "call_allocs" stays flat), with
    every result right.  MV2AMD_POOL=0 (a hipMalloc / hipFree per call, round 4's behaviour)
    allocates on every round; the OSU-style latency of the 64 KiB derived MPI_Bcast is recorded
    for both (MV2AMD_TEST_RECORD: a JSON file the numbers are appended to)."""
    lat = {}
    # "1c": the pool with its idle cap at 1 byte (MV2AMD_POOL_IDLE_MAX): every block goes back to HIP
    # when it is returned, so warm calls allocate again and the trims are counted
    for pool in ("1", "0", "1c"):
        case = {"id": f"dna{pool}", "kind": "derived_no_alloc", "nblocks": 4096, "rounds": 10, "lat_iters": 200}
        (tmp_path / f"p{pool}").mkdir()
        env = {"MV2AMD_POOL": pool[0], **({"MV2AMD_POOL_IDLE_MAX": "1"} if pool == "1c" else {})}
        res = run_workers(n, [case], tmp_path / f"p{pool}", extra_env=env)
        got = [res(case["id"], r) for r in range(n)]
        for r in range(n):
            assert got[r][0] == 0, f"rank {r}: wrong results with MV2AMD_POOL={pool}"
            if pool == "1":
                assert got[r][1] == 0, f"rank {r}: {got[r][1]} device allocations inside warm calls"
                assert got[r][3] == 0, f"rank {r}: idle blocks trimmed under the default cap"
            elif pool == "1c":
                assert got[r][1] > 0 and got[r][3] > 0, f"rank {r}: allocations {got[r][1]}, trims {got[r][3]}"
            else:
                assert got[r][1] > 0
        lat[f"pool={pool}"] = round(float(np.mean([g[2] for g in got])), 2)
    rec = os.environ.get("MV2AMD_TEST_RECORD")
    if rec:
        with open(rec, "a") as f:
            f.write(json.dumps({"test": "derived MPI_Bcast 64 KiB (MPI_Type_vector(4096,4,8,MPI_FLOAT)) OSU latency us",
                                "ranks": n, **lat}) + "\n")


SOAK = [  # (ranks, calls, seed, environment, ranks per emulated node)
    (2, 16000, 11, {}, None), (4, 10000, 12, {}, None), (8, 5000, 13, {}, None),
    # the full-release fallback a node adopts when the light release fails its self-test
    (3, 5000, 14, {"MV2AMD_LIGHT_RELEASE": "0"}, None),
    # small pipeline rounds and a narrow one-shot limit: many rounds and slot turns per call
    (4, 4000, 15, {"MV2AMD_PIPE_GRID": "64", "MV2AMD_PIPE_SUB": str(16 << 10), "MV2AMD_ONESHOT_MAX": str(16 << 10)}, None),
    # point-to-point on the copy engines instead of the copy kernels
    (2, 4000, 16, {"MV2AMD_P2P_KERNEL_COPY": "0"}, None),
    # two emulated nodes: two-level collectives, leaders over TCP
    (4, 1500, 17, {}, 2),
    # two nodes of four: the most processes the GPU runs at once (DESIGN.md §5 "Ranks per GPU"),
    # the 4 MiB calls on the leaders' ring that failed at 12 processes
    (8, 1000, 18, {}, 4),
]


@pytest.mark.timeout(400)
@pytest.mark.parametrize("n,calls,seed,env,ppn", SOAK)
def test_soak_thousands_of_calls(n, calls, seed, env, ppn, tmp_path):
    """mp_gpu_worker.soak: thousands of blocking / nonblocking / stream-ordered collectives and
    point-to-point rings back to back on the same buffers, every result checked against its
    closed form (a visibility hazard that strikes once in thousands of calls
    survives a suite of short tests), with the protocol settings a node may adopt.
    MV2AMD_SOAK_CALLS scales the count for a long run."""
    calls = int(os.environ.get("MV2AMD_SOAK_CALLS", calls))
    case = {"id": "soak", "kind": "soak", "calls": calls, "seed": seed}
    res = run_workers(n, [case], tmp_path, timeout=380, extra_env=env, ppn=ppn)
    for r in range(n):
        wrong, made, first = (int(v) for v in res(case["id"], r)[:3])
        assert made == calls and wrong == 0, f"rank {r}: {wrong} wrong calls of {made}, the first at {first}"


@pytest.mark.parametrize("n", [1, 2, 3])
def test_argument_checks_follow_the_reference(n, tmp_path):
    """The buffer checks of the reference's MPI layer (mpierrs.h MPIR_ERRTEST_ALIAS_COLL,
    *_INPLACE, USERBUFFER), uncommitted derived types and MPI_Pack's space check return the
    reference's error class on every rank, before any rank enters a collective: one valid
    MPI_Allreduce afterwards completes with the right sums (mp_gpu_worker.arg_checks)."""
    case = {"id": "args", "kind": "arg_checks"}
    res = run_workers(n, [case], tmp_path)
    for r in range(n):
        got = res(case["id"], r)
        pairs, bad = got[:-1].reshape(-1, 2), got[-1]
        wrong = [(i, int(g), int(w)) for i, (g, w) in enumerate(pairs) if g != w]
        assert not wrong, f"rank {r}: (call, got, want) {wrong}"
        assert bad == 0, f"rank {r}: the valid MPI_Allreduce after the refused calls is wrong"


def test_hw_queue_limit_reported_when_too_late(tmp_path):
    """Ranks sharing a GPU ask HIP for 2 hardware queues per process before HIP starts (world.cpp
    limit_hw_queues_if_shared: five ranks with 4 queues each starved a kernel for 30 s, r04f).
    When a host framework has already started HIP the setting cannot act; MPI_Init then reports it
    as too late (negative hw_queues_set) instead of claiming it lowered the queues."""
    got = {}
    for first in ("0", "1"):
        (tmp_path / first).mkdir()
        res = run_workers(2, [{"id": "ti", "kind": "tiling_info"}], tmp_path / first,
                          extra_env={"MV2AMD_TEST_HIP_FIRST": first, "GPU_MAX_HW_QUEUES": "4"})
        got[first] = [int(res("ti", r).view(np.int64)[8]) for r in range(2)]
    assert got["0"] == [2, 2], got
    assert got["1"] == [-2, -2], got


def test_absent_peer_is_reported_not_hung(tmp_path):
    """A collective that one rank never enters: the other rank's device wait runs out after
    MV2AMD_TIMEOUT_S, its MPI_Allreduce returns MPI_ERR_OTHER (MPI_ERRORS_RETURN) instead of hanging,
    and the report names what was awaited -- the epoch, the flags seen, the launch that waited
    (call number and epochs), the waited slot as a copy re-reads it from memory (the absent rank's
    older than the epoch), and where the absent rank's host is (coll.cpp check_err_word).  Both
    ranks then finalize normally."""
    # the host barriers share the timeout: the absent rank reaches MPI_Finalize's after 4.5 s, once the
    # other rank's 3 s device wait has been reported, and well within that rank's 3 s barrier wait
    case = {"id": "absent", "kind": "peer_absent", "absent": 1, "sleep": 4.5}
    got = run_workers(2, [case], tmp_path, extra_env={"MV2AMD_TIMEOUT_S": "3"}, expect_fail=True)
    assert [rc for rc, _ in got] == [0, 0], got
    assert int(np.load(tmp_path / "out" / "absent_r0.npy")[0]) == 15  # MPI_ERR_OTHER
    log = got[0][1]
    assert "device collective timed out waiting for a peer" in log, log[-3000:]
    import re
    m0 = re.search(r"waited for epoch (\d+) from ranks 0x3; flags seen: r0=(\d+) r1=(\d+)", log)
    assert m0, log[-3000:]
    ep, f0, f1 = (int(v) for v in m0.groups())
    assert f0 >= ep > f1
    launches = re.search(r"last launches with flag epochs \(call:epochs, <- the waiting one\):(.*)", log)
    waiting = [(int(a), int(b)) for a, b in re.findall(r"(\d+)-(\d+)(?:\(caller's stream\))?<-", launches.group(1))] \
        if launches else []
    assert len(waiting) == 1 and waiting[0][0] <= ep <= waiting[0][1], log[-3000:]
    now = re.search(r"the waited slot now \(host copy\): r0=(\d+) r1=(\d+)", log)
    assert now and int(now.group(1)) >= ep > int(now.group(2)), log[-3000:]
    assert "late peer: local rank 1" in log, log[-3000:]
