"""Several nodes, emulated on the GPU box: n ranks split node-major into
n / ppn nodes, each with its own control segment and IPC world, the node leaders linked over
TCP (runtime/internode.cpp).  Results are checked bit-exactly against a restatement of
MVAPICH2's two-level structure built from the oracle: node step = the oracle's one-node
algorithm for the node's ranks (the small-message shortcuts, and 16-ppn table entries, whose
intra function the one-node selection reads too) or the 2-ppn table entry's reduce_shmem,
inter-node step = the table's recursive doubling or pt2pt_rs over the node leaders (the inter step
of MPIR_Allreduce_two_level_MV2 / topo-aware hierarchical, allreduce_osu.c:360-630, :633-1054,
:1750-1780, :2215) or binomial reduce (reduce_osu.c:425) over the node leaders, every uop an
oracle op-loop call.  Allreduce from 2 MiB is the flat ring over every rank, and where the tables
name it the flat pt2pt_rs / pt2pt_rd over every rank (expected_allreduce); reduce-scatter is
MPIR_Reduce_scatter_MV2's flat selection over every rank (red_scat_osu.c:1771-1900)."""
import json
from pathlib import Path

import numpy as np
import pytest

from mvapich2_amd.consts import OPS, TYPES
from oracle import oracle
from tests import ref_user
from tests.helpers import as_bytes, assert_bytes_equal
from tests.test_gpu_collectives_mp import inputs, run_workers

pytestmark = pytest.mark.gpu


def uop(tmp, acc, count, t, op):
    """uop(tmp, recv) of the reference: recv = tmp (+) recv, the C op loop"""
    out = acc.copy()
    assert oracle.reduce_local(tmp, out, count, TYPES[t][0], OPS[op]) == 0
    return out


def rd_leaders(parts, count, t, op):
    """MPIR_Allreduce_pt2pt_rd_MV2 over the leaders (allreduce_osu.c:455-600), commutative form"""
    n = len(parts)
    acc = [p.copy() for p in parts]
    pof2 = 1
    while pof2 * 2 <= n:
        pof2 *= 2
    rem = n - pof2
    for r in range(1, 2 * rem, 2):
        acc[r] = uop(acc[r - 1], acc[r], count, t, op)
    newrank = {r: (r // 2 if r < 2 * rem else r - rem) for r in range(n) if not (r < 2 * rem and r % 2 == 0)}
    mask = 1
    while mask < pof2:
        snap = [a.copy() for a in acc]
        for r, nr in newrank.items():
            nd = nr ^ mask
            dst = nd * 2 + 1 if nd < rem else nd + rem
            acc[r] = uop(snap[dst], acc[r], count, t, op)
        mask <<= 1
    for r in range(0, 2 * rem, 2):
        acc[r] = acc[r + 1].copy()
    return acc


def binomial_leaders(parts, count, t, op, root):
    """MPIR_Reduce_binomial_MV2 over the leaders to node `root`, commutative form"""
    n = len(parts)
    acc = {rel: parts[(rel + root) % n].copy() for rel in range(n)}
    mask = 1
    while mask < n:
        for rel in range(0, n, 2 * mask):
            if rel | mask < n:
                acc[rel] = uop(acc[rel | mask], acc[rel], count, t, op)
        mask <<= 1
    return acc[0]


def ring_flat(sends, count, t, op):
    """MPIR_Allreduce_pt2pt_ring_MV2 over every rank of the job (allreduce_osu.c:3916-3968): chunk c
    = x_c (+) x_{c+1} (+) ... (+) x_{c-1}, the accumulator inout (uop(comp_chunk, recv_chunk))"""
    n = len(sends)
    cc = count // n
    cb = cc * TYPES[t][3]
    out = np.empty(n * cb, dtype=np.uint8)
    for c in range(n):
        acc = sends[c][c * cb:(c + 1) * cb].copy()
        for j in range(1, n):
            acc = uop(sends[(c + j) % n][c * cb:(c + 1) * cb].copy(), acc, cc, t, op)
        out[c * cb:(c + 1) * cb] = acc
    return out


# the multi-node allreduce tables MVAPICH2 falls back to (allreduce_tuning.c default branch,
# tuning/allreduce/nemesis_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{1,2,16}ppn.h), as data generated from
# the headers by tests/golden/gen_mn_allreduce_tables.py
_TABLES = json.loads((Path(__file__).parent / "golden" / "mn_allreduce_tables.json").read_text())
_INTRA = {"h": "reduce_shmem", "p": "reduce_p2p", "s": "pt2pt_rs", "d": "pt2pt_rd"}


def table_cell(ppn, n, nbytes):
    """MPIR_Allreduce_index_tuned_intra_MV2's table step (allreduce_osu.c:3200-3290): ("2l", inter,
    intra) for a two-level entry, ("flat", algorithm, None) for a flat one (multicast -> pt2pt_rd).
    comm_size_index: the entry of floor_pof2(n), clamped to the table's first and last entries;
    one rank per node: a two-level entry is its leaders' function over every rank; 16 ppn, first
    entry: intra "node" (the node's one-node selection reads the same entry)."""
    tab = _TABLES["1ppn" if ppn <= 1 else "2ppn" if ppn == 2 else "16ppn"]
    if n > tab[-1]["numproc"]:
        ci = len(tab) - 1
    else:
        p, ci = 1 << (n.bit_length() - 1), 0
        while p > tab[0]["numproc"]:
            p, ci = p >> 1, ci + 1
    e = tab[ci]
    idx = min(17, max(0, nbytes.bit_length() - 1))
    fn = "pt2pt_rs" if e["inter"][idx] == "s" else "pt2pt_rd"
    if e["two_level"][idx] != "1" or ppn <= 1:
        return "flat", fn, None
    return "2l", fn, "node" if ppn >= 3 and ci == 0 else _INTRA[e["intra"][idx]]


def table_entry(ppn, n, nbytes, knobs=None):
    """("2l", inter) for a two-level entry or ("flat", algorithm) of MVAPICH2's tables across nodes"""
    return table_cell(ppn, n, nbytes)[:2]


def expected_allreduce(sends, count, t, op, ppn, in_place=False):
    """per-rank results of MPI_Allreduce across nodes, by the selection coll.cpp mn_allreduce
    restates: flat ring from 2 MiB (remainder, IN_PLACE and count < n: the wrapper's flat pt2pt_rs
    over every rank), the small-message shortcuts' two-level order up to 2 KiB, then the tables'
    flat pt2pt_rs / pt2pt_rd or two-level entry"""
    n = len(sends)
    rs = oracle.ALGOS.index("pt2pt_rs")
    if count * TYPES[t][2] >= 2 << 20 and (in_place or count < n):  # the wrapper's pt2pt_rs
        main = (count // n) * n if in_place else 0
        if not main or main == count:
            return oracle.allreduce([x.copy() for x in sends], count, TYPES[t][0], OPS[op], algo=rs)
        # IN_PLACE: the ring body's own pt2pt_rs on (count / n) * n elements, then the remainder's
        ext = TYPES[t][3]
        head = oracle.allreduce([x[:main * ext].copy() for x in sends], main, TYPES[t][0], OPS[op], algo=rs)
        tail = oracle.allreduce([x[main * ext:].copy() for x in sends], count - main, TYPES[t][0], OPS[op], algo=rs)
        return [np.concatenate([head[r], tail[r]]) for r in range(n)]
    if count * TYPES[t][2] >= 2 << 20 and count >= n and not in_place:
        main = ring_flat(sends, count, t, op)
        rem = count % n
        if not rem:
            return [main] * n
        tails = [x[len(main):].copy() for x in sends]
        tail = oracle.allreduce(tails, rem, TYPES[t][0], OPS[op], algo=rs)
        return [np.concatenate([main, tail[r]]) for r in range(n)]
    nbytes = count * TYPES[t][2]
    if nbytes > 2048:  # the topology-aware shortcut up to 2 KiB, then the tables
        kind, fn, intra = table_cell(ppn, n, nbytes)
        if kind == "flat":
            return oracle.allreduce([x.copy() for x in sends], count, TYPES[t][0], OPS[op],
                                    algo=oracle.ALGOS.index(fn))
        return two_level(sends, count, t, op, ppn, inter=fn, intra=intra)
    return two_level(sends, count, t, op, ppn)


# MPIR_Reduce_scatter_MV2's default table (red_scat_tuning.c:214-287): numproc, then the inclusive
# upper bounds of basic / recursive halving / pairwise; the ring beyond, and from
# MV2_RED_SCAT_RING_ALGO_THRESHOLD (131072 B) whatever the entry (red_scat_osu.c:1859-1871)
_RS_TABLE = [(8, 256, 16384, 65536), (16, 64, 65536, 65536), (32, 64, 131072, 131072), (64, 1024, 262144, 262144)]


def rs_algo(n, nbytes, via=None):
    if via == "inb":  # MPI_Ireduce_scatter: MPIR_Ireduce_scatter_pairwise
        return "rs_pairwise"
    if via in ("block", "iblock"):  # MPICH's MPIR_(I)reduce_scatter_block_intra (ired_scat_block.c:882-920)
        return "rs_rec_halving" if nbytes < 524288 else "rs_pairwise"
    if nbytes >= 131072:
        return "rs_ring"
    row = next((r for r in _RS_TABLE if n <= r[0]), _RS_TABLE[-1])
    return "rs_basic" if nbytes <= row[1] else "rs_rec_halving" if nbytes <= row[2] else \
        "rs_pairwise" if nbytes <= row[3] else "rs_ring"


def expected_reduce_scatter(sends, counts, t, op, ppn, via=None):
    """every rank's block of MPI_Reduce_scatter across nodes, concatenated: the algorithm of the
    table over every rank; basic = MPIR_Reduce_MV2 to rank 0 over the whole job (the two-level
    helper: each node's reduce to its local rank 0, binomial over the leaders) + scatter"""
    n, total = len(sends), sum(counts)
    algo = rs_algo(n, total * TYPES[t][2], via)
    if algo == "rs_basic":
        parts = [oracle.reduce_ref([x.copy() for x in sends[j * ppn:(j + 1) * ppn]], total, TYPES[t][0], OPS[op], 0)
                 for j in range(n // ppn)]
        return binomial_leaders(parts, total, t, op, 0)
    return oracle.reduce_scatter_ref([x.copy() for x in sends], counts, TYPES[t][0], OPS[op],
                                     algo=oracle.ALGOS.index(algo))


# the multi-node reduce tables (reduce_tuning.c:1563-1649, tuning/reduce/
# gen2{_cma}_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{1,2,16}ppn.h), generated from the headers by
# tests/golden/gen_mn_reduce_tables.py
_RTABLES = json.loads((Path(__file__).parent / "golden" / "mn_reduce_tables.json").read_text())
_RALGO = {"b": "binomial", "k": "knomial", "r": "redscat_gather", "i": "knomial", "h": "shmem_linear"}


def _pof2(n):
    return 1 << (n.bit_length() - 1)


def _tindex(nbytes, minsz, size):
    """the message-size index (reduce_osu.c:2556-2586): floor(log2(nbytes / smallest)), clamped"""
    if nbytes < minsz:
        return 0
    if nbytes > minsz << (size - 1):
        return size - 1
    return (nbytes // minsz).bit_length() - 1


def reduce_cell(ppn, n, nbytes, cma=True):
    """MPIR_Reduce_index_tuned_intra_MV2's table step (reduce_osu.c:2516-2620): (two_level, inter
    letter, intra letter, knomial factor).  comm_size_index = log2(floor_pof2(n) / floor_pof2(first
    numproc)) clamped to the table's ends — an index, not a numproc match."""
    tab = _RTABLES[("cma_" if cma else "nocma_") + ("1ppn" if ppn <= 1 else "2ppn" if ppn == 2 else "16ppn")]
    if n < tab[0]["numproc"]:
        ci = 0
    elif n > tab[-1]["numproc"]:
        ci = len(tab) - 1
    else:
        ci = max(0, (_pof2(n) // _pof2(tab[0]["numproc"])).bit_length() - 1)
    e = tab[ci]
    ii, ij = _tindex(nbytes, e["inter_min"], len(e["inter"])), _tindex(nbytes, e["intra_min"], len(e["intra"]))
    return e["two_level"][ii] == "1", e["inter"][ii], e["intra"][ij], e["inter_k"]


def expected_reduce(sends, count, t, op, ppn, root):
    """the root's result of MPI_Reduce across nodes (builtin op): up to 1 KiB the small-message
    shortcut (reduce_osu.c:2508-2514: the two-level helper with MPIR_Reduce_shmem_MV2 in the node and
    binomial over the leaders), else the tables: MPIR_Reduce_two_level_helper_MV2 (reduce_osu.c:
    2030-2330: the node's intra function to local rank 0 — shmem becomes the intra knomial from the
    32 KiB shmem slot on — then the inter function over the node leaders to the root's node) or the
    inter function flat over every rank (redscat_gather needs count >= pof2, else binomial).  Every
    step is the oracle's forced algorithm."""
    n, nbytes, ext = len(sends), count * TYPES[t][2], TYPES[t][3]
    nodes, rnode = n // ppn, root // ppn
    two, inter, intra, _k = (True, "b", "h", 4) if nbytes <= 1024 else reduce_cell(ppn, n, nbytes)

    def run(xs, algo, r):
        return oracle.reduce_ref([x.copy() for x in xs], count, TYPES[t][0], OPS[op], r,
                                 algo=oracle.ALGOS.index(_RALGO[algo]))
    if two:
        ia = "k" if intra == "h" and count * ext >= 32768 else intra
        parts = [run(sends[j * ppn:(j + 1) * ppn], ia, 0) if ppn > 1 else sends[j].copy() for j in range(nodes)]
        return run(parts, inter, rnode) if nodes > 1 else parts[0]
    algo = "b" if inter == "r" and count < _pof2(n) else inter
    return run(sends, algo, root)


def node_step(xs, count, t, op, intra, knobs=None):
    """the leader's partial after a two-level entry's intra-node function over the node's ranks
    (MPIR_Allreduce_two_level_MV2 :1727-1745)"""
    if intra == "node":  # the node's own one-node selection
        return oracle.allreduce_ref(xs, count, TYPES[t][0], OPS[op], knobs=knobs)[0]
    if intra == "reduce_p2p":  # MPIR_Reduce_MV2 to local rank 0
        return oracle.reduce_ref(xs, count, TYPES[t][0], OPS[op], 0)
    algo = "shmem_linear" if intra == "reduce_shmem" else intra
    return oracle.allreduce(xs, count, TYPES[t][0], OPS[op], algo=oracle.ALGOS.index(algo))[0]


def two_level(sends, count, t, op, ppn, inter="pt2pt_rd", intra="node", knobs=None):
    """MPIR_Allreduce_two_level_MV2: node step (node_step), the leaders' inter algorithm, node
    broadcast"""
    nodes = len(sends) // ppn
    parts = [node_step([x.copy() for x in sends[j * ppn:(j + 1) * ppn]], count, t, op, intra, knobs)
             for j in range(nodes)]
    if inter == "pt2pt_rd":
        lead = rd_leaders(parts, count, t, op)
    else:
        lead = oracle.allreduce(parts, count, TYPES[t][0], OPS[op], algo=oracle.ALGOS.index(inter))
    return [lead[r // ppn] for r in range(len(sends))]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,ppn", [(4, 2), (6, 2), (3, 1), (8, 4), (6, 3), (4, 1)])
def test_two_level_collectives_across_nodes(n, ppn, tmp_path):
    nodes = n // ppn
    cases, seed = [], 300
    for t, op, count in (("MPI_FLOAT", "MPI_SUM", 10), ("MPI_FLOAT", "MPI_SUM", 300), ("MPI_DOUBLE", "MPI_MAX", 200),
                         ("MPI_FLOAT", "MPI_SUM", 70001), ("MPI_INT", "MPI_SUM", 100003),
                         ("MPI_DOUBLE_INT", "MPI_MAXLOC", 5000), ("MPI_UNSIGNED_CHAR", "MPI_BXOR", 4099)):
        cases.append({"id": f"ma{seed}", "kind": "allreduce", "type": t, "op": op, "count": count, "seed": seed})
        seed += 1
    # from 2 MiB (MV2_ALLREDUCE_RING_ALGO_THRESHOLD) the flat ring over every rank; the remainder
    # (count % n elements) takes the two-level order
    for t, op, count in (("MPI_FLOAT", "MPI_SUM", 840 * 1000), ("MPI_FLOAT", "MPI_SUM", 840 * 1000 + 5),
                         ("MPI_DOUBLE", "MPI_SUM", 300001)):
        cases.append({"id": f"mR{seed}", "kind": "allreduce", "type": t, "op": op, "count": count, "seed": seed})
        seed += 1
    for count in (600000, 600005, 70001):  # IN_PLACE: from 2 MiB the wrapper's pt2pt_rs over every rank
        cases.append({"id": f"mP{seed}", "kind": "allreduce_inplace", "type": "MPI_FLOAT", "op": "MPI_SUM",
                      "count": count, "seed": seed})
        seed += 1
    # nonblocking across nodes: MVAPICH2's nonblocking schedules are flat over the job (Iallreduce =
    # Ireduce to rank 0 + Ibcast, Ireduce = binomial); they complete at initiation here
    for t, count in (("MPI_INT", 5000), ("MPI_FLOAT", 5000), ("MPI_FLOAT", 70001), ("MPI_DOUBLE", 30)):
        cases.append({"id": f"mi{seed}", "kind": "iallreduce", "type": t, "op": "MPI_SUM", "count": count,
                      "seed": seed})
        seed += 1
    for count, root in ((1000, n - 1), (70001, 1 % n)):
        cases.append({"id": f"mj{seed}", "kind": "ireduce", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": count,
                      "seed": seed, "root": root})
        seed += 1
    for t, op, count, root in (("MPI_FLOAT", "MPI_SUM", 1000, n - 1), ("MPI_INT", "MPI_SUM", 70001, 1 % n),
                               ("MPI_DOUBLE", "MPI_MIN", 300, 0)):
        cases.append({"id": f"mr{seed}", "kind": "reduce", "type": t, "op": op, "count": count, "seed": seed,
                      "root": root})
        seed += 1
    # above 1 KiB the multi-node reduce tables (reduce_osu.c:2516-2660): per size the two-level helper
    # with its intra (shmem / binomial / intra knomial) and inter (binomial / knomial / redscat_gather)
    # functions, or one of them flat over every rank (reduce_cell); fp SUM and tie-laden MAX make the
    # operand order visible
    for t, op, count, root, ties in (("MPI_FLOAT", "MPI_SUM", 520, 0, False), ("MPI_FLOAT", "MPI_SUM", 1030, n - 1, False),
                                     ("MPI_FLOAT", "MPI_SUM", 2050, 1 % n, False), ("MPI_DOUBLE", "MPI_SUM", 2049, n - 1, False),
                                     ("MPI_FLOAT", "MPI_SUM", 16400, 0, False), ("MPI_DOUBLE", "MPI_MAX", 1025, n // 2, True),
                                     ("MPI_FLOAT", "MPI_SUM", 40000, n - 1, False)):
        cases.append({"id": f"mq{seed}", "kind": "reduce", "type": t, "op": op, "count": count, "seed": seed,
                      "root": root, "ties": ties})
        seed += 1
    for count, root in ((70001, n - 1), (1000, 1 % n), (5, 0)):
        cases.append({"id": f"mb{seed}", "kind": "bcast", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": count,
                      "seed": seed, "root": root})
        seed += 1
    # 4-8 KiB: the 2-ppn table's numproc 4 entry is two-level (reduce_shmem + recursive doubling);
    # signed zeros and NaN payloads make the operand order visible in MAX / MIN
    for t, op, count in (("MPI_DOUBLE", "MPI_MAX", 600), ("MPI_FLOAT", "MPI_MIN", 1500)):
        cases.append({"id": f"mt{seed}", "kind": "allreduce", "type": t, "op": op, "count": count, "seed": seed,
                      "ties": True})
        seed += 1
    # reduce-scatter over every rank: basic (<= 256 B), recursive halving, pairwise, ring (>= 128 KiB)
    for t, op, per, ties in (("MPI_FLOAT", "MPI_SUM", 7, False), ("MPI_DOUBLE", "MPI_MAX", 150, True),
                             ("MPI_FLOAT", "MPI_SUM", 1500, False), ("MPI_FLOAT", "MPI_SUM", 12000, False)):
        counts = [per + (r % 2) for r in range(n)]
        cases.append({"id": f"ms{seed}", "kind": "reduce_scatter", "type": t, "op": op, "recvcounts": counts,
                      "count": sum(counts), "seed": seed, "ties": ties})
        seed += 1
    # MPI_Ireduce_scatter across nodes: its own flat schedule (MPIR_Ireduce_scatter_MV2 -> pairwise)
    cases.append({"id": f"mn{seed}", "kind": "reduce_scatter", "type": "MPI_FLOAT", "op": "MPI_SUM", "via": "inb",
                  "recvcounts": [3000 + r for r in range(n)], "count": sum(3000 + r for r in range(n)), "seed": seed})
    seed += 1
    # ragged with empty blocks: every other rank receives nothing
    for t, op, per in (("MPI_FLOAT", "MPI_SUM", 1000), ("MPI_DOUBLE", "MPI_MIN", 40000)):
        counts = [0 if r % 2 == 0 else per + r for r in range(n)]
        cases.append({"id": f"mz{seed}", "kind": "reduce_scatter", "type": t, "op": op, "recvcounts": counts,
                      "count": sum(counts), "seed": seed})
        seed += 1
    for t, op, per in (("MPI_INT", "MPI_SUM", 7001), ("MPI_FLOAT", "MPI_SUM", 100)):
        counts = [per + (r % 3) for r in range(n)]
        cases.append({"id": f"ms{seed}", "kind": "reduce_scatter", "type": t, "op": op, "recvcounts": counts,
                      "count": sum(counts), "seed": seed})
        seed += 1
    # x87 long double across nodes: host-evaluated in 80-bit on the same schedules (mpi/user_coll.cpp)
    for kind, op, count in (("allreduce", "MPI_SUM", 100), ("allreduce", "MPI_SUM", 70001),
                            ("allreduce", "MPI_MAX", 1000), ("allreduce", "MPI_SUM", 140001)):
        cases.append({"id": f"mx{seed}", "kind": kind, "type": "MPI_LONG_DOUBLE", "op": op, "count": count,
                      "seed": seed})
        seed += 1
    cases.append({"id": f"mx{seed}", "kind": "reduce", "type": "MPI_LONG_DOUBLE", "op": "MPI_SUM", "count": 30001,
                  "seed": seed, "root": n - 1})
    seed += 1
    xc = [3000 + r for r in range(n)]
    cases.append({"id": f"mx{seed}", "kind": "reduce_scatter", "type": "MPI_LONG_DOUBLE", "op": "MPI_SUM",
                  "recvcounts": xc, "count": sum(xc), "seed": seed})
    seed += 1
    for count in (1000, 100003):
        cases.append({"id": f"mg{seed}", "kind": "allgather", "type": "MPI_CHAR", "op": "MPI_SUM", "count": count,
                      "seed": seed})
        seed += 1
    res = run_workers(n, cases, tmp_path, ppn=ppn)
    for case in cases:
        k, cid, t, count = case["kind"], case["id"], case["type"], case["count"]
        sends = [inputs(case, r).view(np.uint8).ravel().copy() for r in range(n)]
        if k == "iallreduce":
            want = oracle.iallreduce_ref(sends, count, TYPES[t][0], OPS[case["op"]])
            for r in range(n):
                assert_bytes_equal(res(cid, r), want[r], t, count, f"{cid} {t} iallreduce rank {r}")
        elif k == "ireduce":
            want = oracle.ireduce_ref(sends, count, TYPES[t][0], OPS[case["op"]], case["root"])
            assert_bytes_equal(res(cid, case["root"]), want, t, count, f"{cid} ireduce root {case['root']}")
        elif k in ("allreduce", "iallreduce", "allreduce_inplace"):
            want = expected_allreduce(sends, count, t, case["op"], ppn, in_place=k == "allreduce_inplace")
            for r in range(n):
                assert_bytes_equal(res(cid, r), want[r], t, count, f"{cid} {t} {case['op']} rank {r}")
        elif k == "reduce":
            want = expected_reduce(sends, count, t, case["op"], ppn, case["root"])
            assert_bytes_equal(res(cid, case["root"]), want, t, count, f"{cid} reduce root {case['root']}")
        elif k == "reduce_scatter":  # MPIR_Reduce_scatter_MV2 flat over every rank
            counts = case["recvcounts"]
            full = expected_reduce_scatter(sends, counts, t, case["op"], ppn, case.get("via"))
            ext = TYPES[t][3]
            off = 0
            for r in range(n):
                blk = full[off * ext:(off + counts[r]) * ext]
                assert_bytes_equal(res(cid, r), blk, t, counts[r], f"{cid} reduce_scatter rank {r}")
                off += counts[r]
        elif k == "bcast":
            want = as_bytes(inputs(case, case["root"]))
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)
        elif k == "allgather":
            want = np.concatenate([as_bytes(inputs(case, r)) for r in range(n)])
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,ppn", [(6, 3), (8, 4), (4, 2), (8, 2)])
def test_two_level_table_entries_across_nodes(n, ppn, tmp_path):
    """With the small-message shortcuts off (MV2_ENABLE_TOPO_AWARE_COLLECTIVES=0,
    MV2_ENABLE_SKIP_TUNING_TABLE_SEARCH=0) small allreduces read the tables' two-level entries: at
    >= 3 ranks per node the 16-ppn entry's intra function (reduce_shmem, or reduce_p2p = the node's
    MPIR_Reduce_MV2 to local rank 0 from 256 B) and pt2pt_rs over the leaders (recursive doubling
    for count < pof2); at 2 ranks per node the 2-ppn entry's reduce_shmem and recursive doubling."""
    env = {"MV2_ENABLE_TOPO_AWARE_COLLECTIVES": "0", "MV2_ENABLE_SKIP_TUNING_TABLE_SEARCH": "0"}
    k = oracle.default_knobs(enable_topo=0, enable_skip_search=0)
    cases, seed = [], 900
    for t, op, count, ties in (("MPI_FLOAT", "MPI_SUM", 100, False), ("MPI_DOUBLE", "MPI_MAX", 50, True),
                               ("MPI_FLOAT", "MPI_SUM", 60, False), ("MPI_FLOAT", "MPI_MIN", 60, True),
                               ("MPI_INT", "MPI_SUM", 3, False), ("MPI_DOUBLE", "MPI_MAX", 1, True),
                               # 64-127 B: the 2-ppn numproc 8 entry's intra function is pt2pt_rs
                               ("MPI_FLOAT", "MPI_MIN", 20, True), ("MPI_FLOAT", "MPI_SUM", 31, False)):
        cases.append({"id": f"mk{seed}", "kind": "allreduce", "type": t, "op": op, "count": count, "seed": seed,
                      "ties": ties})
        seed += 1
    res = run_workers(n, cases, tmp_path, ppn=ppn, extra_env=env)
    for case in cases:
        cid, t, count = case["id"], case["type"], case["count"]
        sends = [inputs(case, r).view(np.uint8).ravel().copy() for r in range(n)]
        kind, fn, intra = table_cell(ppn, n, count * TYPES[t][2])
        assert kind == "2l", (cid, kind, fn)
        want = two_level(sends, count, t, case["op"], ppn, inter=fn, intra=intra, knobs=k)
        for r in range(n):
            assert_bytes_equal(res(cid, r), want[r], t, count, f"{cid} {t} {case['op']} rank {r}")


def _ufn(a, b):
    """the workers' user op: inout = 2 in + 3 inout (int32, wrapping; neither commutative nor associative)"""
    return (a.astype(np.int64) * 2 + b.astype(np.int64) * 3).astype(np.int32)


def user_allreduce_across(xs, commute, count, ppn):
    """MPI_Allreduce with a user op across nodes (coll.cpp mn_host_schedule): non-commutative ->
    recursive doubling over every rank; commutative -> mn_select's schedule: the topology-aware
    shortcut up to 2 KiB (node tree, leaders' recursive doubling), a 2-ppn two-level entry
    (reduce_shmem + recursive doubling), else the tables' flat pt2pt_rs, which a user op turns into
    recursive doubling (allreduce_osu.c:802)"""
    n = len(xs)
    F = TYPES["MPI_INT"][0]
    if not commute:
        return ref_user.rd(xs, _ufn, False)
    nbytes = count * 4
    if nbytes >= 2 << 20:  # the ring wrapper over every rank, recursive doubling on the remainder
        main = (count // n) * n
        rest = ref_user.rd([x[main:] for x in xs], _ufn, True)
        return [np.concatenate([ref_user.ring_chunks(xs, _ufn, count), rest[r]]) for r in range(n)]
    if nbytes <= 2048 and ppn == 1:
        parts = [x.copy() for x in xs]
    elif nbytes <= 2048:
        parts = [ref_user.allreduce(xs[j * ppn:(j + 1) * ppn], _ufn, True, F, count)[0] for j in range(n // ppn)]
    else:
        kind, fn = table_entry(ppn, n, nbytes)
        if kind == "flat":
            return ref_user.rd(xs, _ufn, True)
        parts = [ref_user.linear(xs[j * ppn:(j + 1) * ppn], _ufn) for j in range(n // ppn)]
    lead = ref_user.rd(parts, _ufn, True)
    return [lead[r // ppn] for r in range(n)]


def user_reduce_across(xs, commute, count, ppn, root):
    """MPI_Reduce with a user op across nodes (coll.cpp mn_host_schedule): non-commutative -> the
    flat binomial; commutative -> the device path's selection (expected_reduce), with a user op's
    flat redscat_gather falling back to binomial (it needs a builtin op, reduce_osu.c:2645-2652) while
    the two-level helper's leaders run the table's function as it is (:2315)"""
    n = len(xs)
    if not commute:
        return ref_user.reduce(xs, _ufn, False, TYPES["MPI_INT"][0], count, root)
    nbytes, nodes = count * 4, n // ppn
    two, inter, intra, k = (True, "b", "h", 4) if nbytes <= 1024 else reduce_cell(ppn, n, nbytes)

    def run(ys, a, r):
        if a == "b":
            return ref_user.binomial(ys, _ufn, r, True)
        if a in "ki":
            return ref_user.knomial(ys, _ufn, r, k)
        if a == "h":
            return ref_user.linear(ys, _ufn)
        return ref_user.redscat_gather(ys, _ufn, count)
    if two:
        ia = "k" if intra == "h" and count * 4 >= 32768 else intra
        parts = [run(xs[j * ppn:(j + 1) * ppn], ia, 0) if ppn > 1 else xs[j].copy() for j in range(nodes)]
        return run(parts, inter, root // ppn) if nodes > 1 else parts[0]
    return run(xs, "b" if inter == "r" else inter, root)


@pytest.mark.timeout(300)
# (ranks, ranks per node, MV2AMD_MN_PROG_MAX): at most 8 processes share the one GPU (DESIGN.md §5
# "Ranks per GPU"), so the schedules of jobs above 8 ranks / 8 nodes run at 8 and 6 ranks with the
# programs' limit lowered to 4
@pytest.mark.parametrize("n,ppn,pm", [(4, 2, 8), (6, 3, 8), (8, 4, 8), (3, 1, 8), (8, 1, 4), (6, 2, 4)])
def test_user_ops_across_nodes(n, ppn, pm, tmp_path):
    """User MPI_Ops across nodes (host-evaluated, mpi/user_coll.cpp): the device path's schedule
    over the job's ranks — two-level (node step, leaders' step) or flat — with operands that travel
    packed over the leaders' links; MPI_Reduce: the two-level helper (node reduce to local rank 0,
    binomial over the leaders) for a commutative op, the flat binomial for a non-commutative one;
    MPI_Reduce_scatter: MPIR_Reduce_scatter_MV2's flat selection (non_comm forms included).  Above
    the programs' limit (8 ranks; 4 in the 8x1 and 6x2 cases) the host evaluates the message
    schedules themselves (user_coll.cpp BigEval: recursive doubling, the ring's own chunk, the
    binomial; leaders' steps over more nodes than the limit; reduce-scatter's basic / recursive
    halving / ring for this rank's block, and the non-commutative reduce-scatter's recursive
    doubling as an expression tree)."""
    cases, seed = [], 700
    for commute in (1, 0):
        for count in (100, 2000, 33) + ((600001,) if commute and n > pm else ()):
            cases.append({"id": f"ua{seed}", "kind": "user_allreduce", "commute": commute, "count": count,
                          "type": "MPI_INT", "seed": seed})
            seed += 1
        for count, root in ((100, n - 1), (3000, 1 % n), (1030, 0), (4100, n - 1), (16400, n // 2)):
            cases.append({"id": f"ur{seed}", "kind": "user_reduce", "commute": commute, "count": count,
                          "type": "MPI_INT", "seed": seed, "root": root})
            seed += 1
        # above the limit: basic (a 24-byte operand, half the blocks empty), halving, ring; the
        # non_comm recursive doubling from its expression tree (user_coll.cpp BigEval::expr)
        for per in (3, 400) if n <= pm else (0, 400, 12000) if commute else (5, 300):
            counts = [per] * n if not commute else [per + (r % 2) for r in range(n)]
            cases.append({"id": f"us{seed}", "kind": "user_reduce_scatter", "commute": commute, "count": sum(counts),
                          "recvcounts": counts, "type": "MPI_INT", "seed": seed})
            seed += 1
    res = run_workers(n, cases, tmp_path, ppn=ppn, extra_env={"MV2AMD_MN_PROG_MAX": str(pm)})
    for case in cases:
        cid, k, count, commute = case["id"], case["kind"], case["count"], bool(case["commute"])
        if k == "user_allreduce":
            xs = [(np.arange(count, dtype=np.int32) + r) % 7 for r in range(n)]
            want = user_allreduce_across(xs, commute, count, ppn)
            for r in range(n):
                assert np.array_equal(res(cid, r).view(np.int32), want[r]), (cid, r)
        elif k == "user_reduce":
            xs = [(np.arange(count, dtype=np.int32) + r) % 7 for r in range(n)]
            root = case["root"]
            want = user_reduce_across(xs, commute, count, ppn, root)
            assert np.array_equal(res(cid, root).view(np.int32), want), (cid, root)
        else:
            counts = case["recvcounts"]
            total = sum(counts)
            xs = [((np.arange(total) + r) % 7).astype(np.int32) for r in range(n)]
            if commute and rs_algo(n, total * 4) == "rs_basic":  # the multi-node reduce to 0 + scatter
                parts = [ref_user.reduce(xs[j * ppn:(j + 1) * ppn], _ufn, True, TYPES["MPI_INT"][0], total, 0)
                         for j in range(n // ppn)] if ppn > 1 else xs
                full = ref_user.binomial(parts, _ufn, 0, True)
                offs = np.cumsum([0] + counts)
                want = [full[offs[r]:offs[r + 1]] for r in range(n)]
            else:
                want = ref_user.reduce_scatter(xs, _ufn, TYPES["MPI_INT"][0], counts, algo=rs_algo(n, total * 4)) \
                    if commute else ref_user.reduce_scatter_noncomm(xs, _ufn, counts)
            for r in range(n):
                assert np.array_equal(res(cid, r).view(np.int32), want[r]), (cid, r)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,ppn", [(4, 2), (3, 1)])
def test_stream_ordered_across_nodes(n, ppn, tmp_path):
    """MPIX_*_enqueue across nodes: the call waits for the caller's stream, runs the blocking
    multi-node schedule and returns complete, so the chain of tests/mp_gpu_worker.py enqueue_seq
    (y = Allreduce(x), z = Allreduce(y) in stream order, Bcast, Reduce_scatter, Allgather, a
    blocking Allreduce between, Reduce MAX to 0) gives the blocking calls' results; capture stays
    refused."""
    F = TYPES["MPI_FLOAT"][0]
    cases = []
    for seed, c in ((511, 1000), (512, (1 << 20) + 5)):
        counts = [c // n + (1 if r < c % n else 0) for r in range(n)]
        cases.append({"id": f"eq{seed}", "kind": "enqueue_seq", "type": "MPI_FLOAT", "count": c, "seed": seed,
                      "recvcounts": counts, "per": c // n})
    res = run_workers(n, cases, tmp_path, ppn=ppn)
    for case in cases:
        c, counts, per = case["count"], case["recvcounts"], case["per"]
        xs = [inputs(case, r).view(np.uint8).ravel().copy() for r in range(n)]
        y = expected_allreduce(xs, c, "MPI_FLOAT", "MPI_SUM", ppn)
        z = expected_allreduce([y[r].copy() for r in range(n)], c, "MPI_FLOAT", "MPI_SUM", ppn)
        rs_full = oracle.reduce_scatter_ref([x.copy() for x in xs], counts, F, OPS["MPI_SUM"])
        ag = np.concatenate([x[:per * 4] for x in xs])
        parts0 = [oracle.reduce_ref([x.copy() for x in xs[j * ppn:(j + 1) * ppn]], c, F, OPS["MPI_MAX"], 0)
                  for j in range(n // ppn)]
        red = binomial_leaders(parts0, c, "MPI_FLOAT", "MPI_MAX", 0)
        for r in range(n):
            got = res(case["id"], r)
            o, parts = 0, {}
            for name, nb in (("y", c * 4), ("z", c * 4), ("xb", c * 4), ("w", c * 4), ("rs", counts[r] * 4),
                             ("ag", per * n * 4), ("r", c * 4), ("w2", c * 4)):
                parts[name] = got[o:o + nb]
                o += nb
            tag = f"{case['id']} rank {r}"
            assert_bytes_equal(parts["y"], y[r], "MPI_FLOAT", c, tag + " y")
            assert_bytes_equal(parts["z"], z[r], "MPI_FLOAT", c, tag + " z")
            assert np.array_equal(parts["xb"], xs[1 % n]), tag + " bcast"
            assert_bytes_equal(parts["w"], y[r], "MPI_FLOAT", c, tag + " blocking w")
            assert_bytes_equal(parts["w2"], y[r], "MPI_FLOAT", c, tag + " w2")
            off = sum(counts[:r]) * 4
            assert_bytes_equal(parts["rs"], rs_full[off:off + counts[r] * 4], "MPI_FLOAT", counts[r], tag + " rs")
            assert np.array_equal(parts["ag"], ag), tag + " allgather"
            if r == 0:
                assert_bytes_equal(parts["r"], red, "MPI_FLOAT", c, tag + " reduce")


@pytest.mark.timeout(200)
def test_mpit_counts_across_nodes(tmp_path):
    """MPI_T across nodes: Allreduce counts MPIR_Allreduce_two_level_MV2 (allreduce_osu.c:1693) and,
    on the node leaders, the leaders' recursive doubling (pt2pt_rd :366); Reduce counts the
    two-level helper (reduce_osu.c:2039) and the leaders' function of the table entry; a 2.4 MB Allreduce the
    flat ring wrapper and ring (:3761, :3898); Reduce_scatter (400 floats over 4 ranks) its flat
    recursive halving (red_scat_osu.c:449)."""
    import json
    n, ppn = 4, 2
    calls = [{"coll": "allreduce", "type": "MPI_FLOAT", "count": 300},
             {"coll": "reduce", "type": "MPI_INT", "count": 2000, "root": n - 1},
             {"coll": "reduce_scatter", "type": "MPI_FLOAT", "count": 100},
             {"coll": "allreduce", "type": "MPI_FLOAT", "count": 600000},  # the flat ring (wrapper, :3761)
             {"coll": "allreduce", "type": "MPI_FLOAT", "count": 70001}]  # 2-ppn table: flat pt2pt_rs
    res = run_workers(n, [{"id": "mpit", "kind": "mpit_counts", "calls": calls}], tmp_path, ppn=ppn)
    # the 8000-byte reduce reads the 2-ppn table: the two-level helper, its leaders' function counted
    # on the leaders (reduce_osu.c:2315 calls it there)
    two, inter, _intra, _k = reduce_cell(ppn, n, 8000)
    assert two
    lead = {"b": "mv2_coll_reduce_binomial", "k": "mv2_coll_reduce_knomial", "r": "mv2_coll_reduce_redscat_gather"}[inter]
    for r in range(n):
        want = {"mv2_coll_allreduce_2lvl": 1, "mv2_coll_reduce_two_level_helper": 1,
                "mv2_coll_reduce_scatter_rec_halving": 1, "mv2_coll_allreduce_pt2pt_ring_wrapper": 1, "mv2_coll_allreduce_pt2pt_ring": 1,
                "mv2_coll_allreduce_shm_rs": 1}
        if r % ppn == 0:
            want.update({"mv2_coll_allreduce_shm_rd": 1, lead: 1})
        got = json.loads(res("mpit", r).tobytes().decode())
        assert {k: v for k, v in got.items() if v} == want, (r, got)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("n,ppn", [(8, 1), (8, 2), (6, 2), (8, 4)])
def test_more_than_eight_ranks_across_nodes(n, ppn, tmp_path):
    """What jobs of more than 8 ranks run, on at most 8 processes (more must not share the one GPU,
    DESIGN.md §5 "Ranks per GPU"): with the programs' limit lowered to 4 (MV2AMD_MN_PROG_MAX) the
    flat pt2pt_rs / pt2pt_rd the tables name over every rank, and the ring wrapper's pt2pt_rs
    remainder, run as the reference's message schedule over the point-to-point channels (coll.cpp
    sched_allreduce, RankChannels); the small-message shortcut's recursive doubling over more node
    leaders than the limit (8x1: LeaderLinks); MPI_Reduce_scatter's schedules over every rank
    (sched_rs_halving / _pairwise / _ring); the nonblocking Iallreduce / Ireduce schedules flat over
    every rank (mn_sched_naive).  (The tables' numproc 16 entries that 10 and 12 ranks select are
    CPU-tested, tests/test_multinode_tables.py.)"""
    cases, seed = [], 1300
    for t, op, count, ties in (("MPI_FLOAT", "MPI_SUM", 10, False), ("MPI_FLOAT", "MPI_SUM", 300, False),
                               ("MPI_FLOAT", "MPI_SUM", 700, False), ("MPI_FLOAT", "MPI_SUM", 1500, False),
                               ("MPI_FLOAT", "MPI_SUM", 5000, False), ("MPI_FLOAT", "MPI_SUM", 70001, False),
                               ("MPI_INT", "MPI_SUM", 100003, False), ("MPI_DOUBLE", "MPI_MAX", 3000, True),
                               ("MPI_FLOAT", "MPI_MIN", 1100, True), ("MPI_DOUBLE_INT", "MPI_MAXLOC", 5000, False),
                               ("MPI_UNSIGNED_CHAR", "MPI_BXOR", 4099, False), ("MPI_DOUBLE", "MPI_SUM", 300001, False),
                               ("MPI_FLOAT", "MPI_SUM", 840 * 1000 + 5, False)):
        cases.append({"id": f"m9{seed}", "kind": "allreduce", "type": t, "op": op, "count": count, "seed": seed,
                      "ties": ties})
        seed += 1
    for count in (600005, 3001):
        cases.append({"id": f"m9{seed}", "kind": "allreduce_inplace", "type": "MPI_FLOAT", "op": "MPI_SUM",
                      "count": count, "seed": seed})
        seed += 1
    # MPI_Reduce: the shortcut, then the tables' helper / flat algorithms (knomial and redscat_gather
    # flat over every rank run their message schedules above 8 ranks, the leaders' above 8 nodes)
    for count, root in ((1000, n - 1), (70001, 1), (1030, 0), (2050, n - 1), (4100, 2), (16400, n - 1), (40000, 0)):
        cases.append({"id": f"m9{seed}", "kind": "reduce", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": count,
                      "seed": seed, "root": root})
        seed += 1
    cases.append({"id": f"m9{seed}", "kind": "bcast", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": 70001,
                  "seed": seed, "root": n - 2})
    seed += 1
    cases.append({"id": f"m9{seed}", "kind": "allgather", "type": "MPI_CHAR", "op": "MPI_SUM", "count": 3001,
                  "seed": seed})
    seed += 1
    # x87 long double (host-evaluated builtin ops): pt2pt_rs's reduce-scatter + allgather, the ring
    # and its remainder, the IN_PLACE split, recursive doubling, MAX ties, the reduce
    for kind, op, count in (("allreduce", "MPI_SUM", 100), ("allreduce", "MPI_SUM", 70001),
                            ("allreduce", "MPI_MAX", 1000), ("allreduce", "MPI_SUM", 140005),
                            ("allreduce_inplace", "MPI_SUM", 140005), ("allreduce", "MPI_SUM", 9)):
        cases.append({"id": f"m9{seed}", "kind": kind, "type": "MPI_LONG_DOUBLE", "op": op, "count": count,
                      "seed": seed})
        seed += 1
    cases.append({"id": f"m9{seed}", "kind": "reduce", "type": "MPI_LONG_DOUBLE", "op": "MPI_SUM", "count": 3001,
                  "seed": seed, "root": n - 1})
    seed += 1
    # the nonblocking schedules, flat over the job: Iallreduce = Ireduce to 0 (redscat_gather above
    # 2 KiB with count >= pof2, else binomial) + Ibcast; Ireduce = binomial
    for t, op, count, ties in (("MPI_INT", "MPI_SUM", 5000, False), ("MPI_FLOAT", "MPI_SUM", 5000, False),
                               ("MPI_FLOAT", "MPI_SUM", 70001, False), ("MPI_DOUBLE", "MPI_SUM", 30, False),
                               ("MPI_DOUBLE", "MPI_MAX", 3000, True)):
        cases.append({"id": f"m9{seed}", "kind": "iallreduce", "type": t, "op": op, "count": count, "seed": seed,
                      "ties": ties})
        seed += 1
    for count, root in ((1000, n - 1), (70001, 1), (7, 0)):
        cases.append({"id": f"m9{seed}", "kind": "ireduce", "type": "MPI_FLOAT", "op": "MPI_SUM", "count": count,
                      "seed": seed, "root": root})
        seed += 1
    # reduce-scatter over every rank as message schedules: basic (<= 64 B at 9-16 ranks: the
    # multi-node reduce + scatter), recursive halving (to 64 KiB), the ring, MPI_Ireduce_scatter's
    # pairwise; ragged counts with empty blocks; signed zeros / NaN payloads under MAX
    for t, op, counts, via, ties in (
            ("MPI_FLOAT", "MPI_SUM", [1] * n, None, False),
            ("MPI_FLOAT", "MPI_SUM", [100 + r for r in range(n)], None, False),
            ("MPI_DOUBLE", "MPI_MAX", [300 + (r % 3) for r in range(n)], None, True),
            ("MPI_FLOAT", "MPI_SUM", [0 if r % 3 == 0 else 500 + r for r in range(n)], None, False),
            ("MPI_FLOAT", "MPI_SUM", [12000 + r for r in range(n)], None, False),
            ("MPI_INT", "MPI_SUM", [0 if r % 2 else 9000 for r in range(n)], None, False),
            ("MPI_FLOAT", "MPI_SUM", [700 + r for r in range(n)], "inb", False),
            ("MPI_FLOAT", "MPI_SUM", [500] * n, "block", False),
            ("MPI_FLOAT", "MPI_SUM", [12000] * n, "iblock", False)):
        case = {"id": f"m9{seed}", "kind": "reduce_scatter", "type": t, "op": op, "recvcounts": counts,
                "count": sum(counts), "seed": seed, "ties": ties}
        if via:
            case["via"] = via
        cases.append(case)
        seed += 1
    res = run_workers(n, cases, tmp_path, ppn=ppn, extra_env={"MV2AMD_MN_PROG_MAX": "4"})
    nodes = n // ppn
    for case in cases:
        k, cid, t, count = case["kind"], case["id"], case["type"], case["count"]
        sends = [inputs(case, r).view(np.uint8).ravel().copy() for r in range(n)]
        if k in ("allreduce", "allreduce_inplace"):
            want = expected_allreduce(sends, count, t, case["op"], ppn, in_place=k == "allreduce_inplace")
            for r in range(n):
                assert_bytes_equal(res(cid, r), want[r], t, count, f"{cid} {t} {case['op']} rank {r}")
        elif k == "iallreduce":
            want = oracle.iallreduce_ref(sends, count, TYPES[t][0], OPS[case["op"]])
            for r in range(n):
                assert_bytes_equal(res(cid, r), want[r], t, count, f"{cid} {t} iallreduce rank {r}")
        elif k == "ireduce":
            want = oracle.ireduce_ref(sends, count, TYPES[t][0], OPS[case["op"]], case["root"])
            assert_bytes_equal(res(cid, case["root"]), want, t, count, f"{cid} ireduce root {case['root']}")
        elif k == "reduce":
            want = expected_reduce(sends, count, t, case["op"], ppn, case["root"])
            assert_bytes_equal(res(cid, case["root"]), want, t, count, f"{cid} reduce root {case['root']}")
        elif k == "bcast":
            want = as_bytes(inputs(case, case["root"]))
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)
        elif k == "reduce_scatter":
            counts, ext = case["recvcounts"], TYPES[t][3]
            full = expected_reduce_scatter(sends, counts, t, case["op"], ppn, case.get("via"))
            offs = np.cumsum([0] + counts) * ext
            for r in range(n):
                assert_bytes_equal(res(cid, r), full[offs[r]:offs[r + 1]], t, counts[r], f"{cid} reduce_scatter rank {r}")
        else:
            want = np.concatenate([as_bytes(inputs(case, r)) for r in range(n)])
            for r in range(n):
                assert np.array_equal(res(cid, r), want), (cid, r)
