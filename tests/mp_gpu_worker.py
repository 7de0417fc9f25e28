"""One rank of the multi-process GPU collective tests (launched by
tests/test_gpu_collectives_mp.py; several ranks may share one GPU).
Runs every case of the spec through the MPI API and saves its result."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402
from tests.helpers import rand_typed  # noqa: E402

WORLD = 0x44000000


def inputs(case, rank):
    rng = np.random.default_rng(case["seed"] * 1000 + rank)
    return rand_typed(case["type"], case["count"], rng, small=case.get("small", False),
                      ties=case.get("ties", False))


def enqueue_seq(L, case, rank, n):
    """On a HIP stream of its own: y = Allreduce(x); z = Allreduce(y) (reads the previous call's
    result in stream order); Bcast(xb) from root 1 % n; Reduce_scatter(x); Allgather(first `per`
    elements of x); then a blocking MPI_Allreduce(x) -> w on the library's stream (must run after
    the queued calls); then Reduce(x, MAX) to root 0 on the stream again.  One host sync at the
    end; the stream is destroyed and one more blocking MPI_Allreduce(x) -> w2 follows.
    Returns the concatenated bytes y | z | xb | w | rs | ag | r | w2."""
    hip = ctypes.CDLL("libamdhip64.so")
    st = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(st)) == 0
    F, SUM, MAX = TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"], OPS["MPI_MAX"]
    c = case["count"]
    x = inputs(case, rank)
    counts = case["recvcounts"]
    per = case["per"]
    sb = m.DeviceBuffer.from_array(x)
    y, z, w, r = (m.DeviceBuffer(c * 4) for _ in range(4))
    xb = m.DeviceBuffer.from_array(x)
    rs, ag = m.DeviceBuffer(max(1, counts[rank]) * 4), m.DeviceBuffer(per * n * 4)
    for b in (y, z, w, r):
        b.upload(np.zeros(c, dtype=np.float32))
    rcs = (ctypes.c_int * n)(*counts)
    s = st.value
    P = ctypes.c_void_p
    assert L.MPIX_Allreduce_enqueue(P(sb.ptr), P(y.ptr), c, F, SUM, WORLD, P(s)) == 0
    assert L.MPIX_Allreduce_enqueue(P(y.ptr), P(z.ptr), c, F, SUM, WORLD, P(s)) == 0
    assert L.MPIX_Bcast_enqueue(P(xb.ptr), c, F, 1 % n, WORLD, P(s)) == 0
    assert L.MPIX_Reduce_scatter_enqueue(P(sb.ptr), P(rs.ptr), rcs, F, SUM, WORLD, P(s)) == 0
    assert L.MPIX_Allgather_enqueue(P(sb.ptr), per, F, P(ag.ptr), per, F, WORLD, P(s)) == 0
    assert L.MPI_Allreduce(sb.ptr, w.ptr, c, F, SUM, WORLD) == 0
    assert L.MPIX_Reduce_enqueue(P(sb.ptr), P(r.ptr), c, F, MAX, 0, WORLD, P(s)) == 0
    # refused: host buffers and user ops cannot be stream-ordered
    hx = np.zeros(4, dtype=np.float32)
    assert L.MPIX_Allreduce_enqueue(P(hx.ctypes.data), P(y.ptr), 4, F, SUM, WORLD, P(s)) != 0
    assert L.MPIX_Allreduce_enqueue(P(sb.ptr), P(y.ptr), 4, F, SUM, WORLD, None) != 0
    # refused: a captured collective on a buffer off a 16-byte boundary (no staging in a graph)
    cap, graph = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(cap)) == 0
    assert hip.hipStreamBeginCapture(cap, 2) == 0  # hipStreamCaptureModeRelaxed
    rc_cap = L.MPIX_Bcast_enqueue(P(xb.ptr + 4), c - 1, F, 0, WORLD, cap)
    assert hip.hipStreamEndCapture(cap, ctypes.byref(graph)) == 0
    if graph.value:
        hip.hipGraphDestroy(graph)
    hip.hipStreamDestroy(cap)
    assert rc_cap != 0
    assert hip.hipStreamSynchronize(st) == 0
    assert L.MPIX_Enqueue_check(WORLD) == 0
    out = [b.download(np.uint8, count=nb) for b, nb in ((y, c * 4), (z, c * 4), (xb, c * 4), (w, c * 4),
                                                       (rs, counts[rank] * 4), (ag, per * n * 4), (r, c * 4))]
    hip.hipStreamDestroy(st)
    # a blocking call after the caller destroyed its stream: the library keeps no handle to it
    w2 = m.DeviceBuffer(c * 4)
    assert L.MPI_Allreduce(sb.ptr, w2.ptr, c, F, SUM, WORLD) == 0
    out.append(w2.download(np.uint8, count=c * 4))
    return np.concatenate(out)


def graph_allreduce(L, case, rank, n):
    """HIP graph capture (graph lane): MPIX_Allreduce_enqueue captured on a stream for each count,
    the graphs instantiated once and replayed `reps` times in an interleaved order with new
    operands each time and a blocking MPI_Allreduce between replays (the host lane); returns
    every replay's result and every blocking result, concatenated."""
    hip = ctypes.CDLL("libamdhip64.so")
    F, SUM = TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]
    P = ctypes.c_void_p
    st = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(st)) == 0
    counts, reps = case["counts"], case["reps"]
    bufs, execs = [], []
    for c in counts:
        sb, rb = m.DeviceBuffer(c * 4), m.DeviceBuffer(c * 4)
        graph, ex = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipStreamBeginCapture(st, 2) == 0  # hipStreamCaptureModeRelaxed
        rc = L.MPIX_Allreduce_enqueue(P(sb.ptr), P(rb.ptr), c, F, SUM, WORLD, st)
        assert hip.hipStreamEndCapture(st, ctypes.byref(graph)) == 0
        assert rc == 0, rc
        assert hip.hipGraphInstantiate(ctypes.byref(ex), graph, None, None, 0) == 0
        bufs.append((sb, rb, graph))
        execs.append(ex)
    out = []
    hb_s, hb_r = m.DeviceBuffer(4096 * 4), m.DeviceBuffer(4096 * 4)
    for k in range(reps):
        for g, c in enumerate(counts):
            sb, rb, _ = bufs[g]
            sb.upload(np.random.default_rng(case["seed"] * 100000 + k * 1000 + g * 10 + rank).standard_normal(c).astype(np.float32))
            assert hip.hipGraphLaunch(execs[g], st) == 0
            assert hip.hipStreamSynchronize(st) == 0
            out.append(rb.download(np.uint8, count=c * 4))
        # the host lane between replays
        hb_s.upload(np.random.default_rng(case["seed"] * 7 + k * 13 + rank).standard_normal(4096).astype(np.float32))
        assert L.MPI_Allreduce(hb_s.ptr, hb_r.ptr, 4096, F, SUM, WORLD) == 0
        out.append(hb_r.download(np.uint8, count=4096 * 4))
    assert L.MPIX_Enqueue_check(WORLD) == 0
    for g, ex in enumerate(execs):
        hip.hipGraphExecDestroy(ex)
        hip.hipGraphDestroy(bufs[g][2])
    hip.hipStreamDestroy(st)
    return np.concatenate(out)


def graph_collectives(L, case, rank, n):
    """HIP graph capture of every stream-ordered collective (graph lane): one capture holds
    MPIX_Reduce_scatter_enqueue, MPIX_Allgather_enqueue, MPIX_Bcast_enqueue, MPIX_Reduce_enqueue
    and MPIX_Allreduce_enqueue back to back, for small (one-shot) and large (pipelined) sizes;
    each graph is replayed `reps` times with new operands, a blocking MPI_Allgather between
    replays (the host lane).  int32 SUM / MAX: exact whatever the order.  Returns the number of
    wrong results."""
    hip = ctypes.CDLL("libamdhip64.so")
    I, SUM, MAX = TYPES["MPI_INT"][0], OPS["MPI_SUM"], OPS["MPI_MAX"]
    P = ctypes.c_void_p
    st = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(st)) == 0
    rb_root, bc_root = 0, 1 % n
    graphs = []
    for c in case["counts"]:  # elements per rank block
        bufs = {k: m.DeviceBuffer(c * n * 4) for k in ("rs_s", "rs_r", "ag_s", "ag_r", "bc", "rd_s", "rd_r", "ar_s", "ar_r")}
        counts = (ctypes.c_int * n)(*([c] * n))
        graph, ex = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipStreamBeginCapture(st, 2) == 0  # hipStreamCaptureModeRelaxed
        rcs = [L.MPIX_Reduce_scatter_enqueue(P(bufs["rs_s"].ptr), P(bufs["rs_r"].ptr), counts, I, SUM, WORLD, st),
               L.MPIX_Allgather_enqueue(P(bufs["ag_s"].ptr), c, I, P(bufs["ag_r"].ptr), c, I, WORLD, st),
               L.MPIX_Bcast_enqueue(P(bufs["bc"].ptr), c, I, bc_root, WORLD, st),
               L.MPIX_Reduce_enqueue(P(bufs["rd_s"].ptr), P(bufs["rd_r"].ptr), c, I, MAX, rb_root, WORLD, st),
               L.MPIX_Allreduce_enqueue(P(bufs["ar_s"].ptr), P(bufs["ar_r"].ptr), c, I, SUM, WORLD, st)]
        assert hip.hipStreamEndCapture(st, ctypes.byref(graph)) == 0
        assert rcs == [0] * 5, rcs
        assert hip.hipGraphInstantiate(ctypes.byref(ex), graph, None, None, 0) == 0
        graphs.append((c, bufs, graph, ex))
    hs, hr = m.DeviceBuffer(64 * 4), m.DeviceBuffer(64 * 4 * n)
    bad = 0

    def pat(r, k, g, cnt):
        return ((np.arange(cnt, dtype=np.int64) * 40503 + r * 977 + k * 131 + g * 7) % 1000003).astype(np.int32)

    for k in range(case["reps"]):
        for g, (c, b, _, ex) in enumerate(graphs):
            b["rs_s"].upload(pat(rank, k, g, c * n))
            b["ag_s"].upload(pat(rank, k, g + 1, c))
            b["bc"].upload(pat(rank, k, g + 2, c) if rank == bc_root else np.full(c, -1, dtype=np.int32))
            b["rd_s"].upload(pat(rank, k, g + 3, c))
            b["ar_s"].upload(pat(rank, k, g + 4, c))
            assert hip.hipGraphLaunch(ex, st) == 0
            assert hip.hipStreamSynchronize(st) == 0
            want_rs = sum(pat(r, k, g, c * n)[rank * c:(rank + 1) * c].astype(np.int64) for r in range(n))
            bad += int(not np.array_equal(b["rs_r"].download(np.int32, count=c), want_rs.astype(np.int32)))
            bad += int(not np.array_equal(b["ag_r"].download(np.int32, count=c * n),
                                          np.concatenate([pat(r, k, g + 1, c) for r in range(n)])))
            bad += int(not np.array_equal(b["bc"].download(np.int32, count=c), pat(bc_root, k, g + 2, c)))
            if rank == rb_root:
                want = np.max(np.stack([pat(r, k, g + 3, c) for r in range(n)]), axis=0)
                bad += int(not np.array_equal(b["rd_r"].download(np.int32, count=c), want))
            want_ar = sum(pat(r, k, g + 4, c).astype(np.int64) for r in range(n)).astype(np.int32)
            bad += int(not np.array_equal(b["ar_r"].download(np.int32, count=c), want_ar))
        # the host lane between replays
        hs.upload(pat(rank, k, 99, 64))
        assert L.MPI_Allgather(hs.ptr, 64, I, hr.ptr, 64, I, WORLD) == 0
        bad += int(not np.array_equal(hr.download(np.int32, count=64 * n),
                                      np.concatenate([pat(r, k, 99, 64) for r in range(n)])))
    assert L.MPIX_Enqueue_check(WORLD) == 0
    for _, _, graph, ex in graphs:
        hip.hipGraphExecDestroy(ex)
        hip.hipGraphDestroy(graph)
    hip.hipStreamDestroy(st)
    return np.array([bad], dtype=np.int64)


def big_case(L, case, rank, n):
    """Full-size BASELINE configs, checked in the worker against closed forms (256 MiB results
    are not shipped back): returns [number of wrong elements]."""
    k = case["kind"]
    F = TYPES["MPI_FLOAT"][0]
    if k == "big_allreduce":  # configs[2]: osu_allreduce fp32 SUM 256 MiB, OMB-style exact pattern
        cnt = case["count"]
        i = np.arange(cnt, dtype=np.int64)
        x = ((i % 100 + 1) * (rank + 1)).astype(np.float32)
        sb, rb = m.DeviceBuffer.from_array(x), m.DeviceBuffer(cnt * 4)
        assert L.MPI_Allreduce(sb.ptr, rb.ptr, cnt, F, OPS["MPI_SUM"], WORLD) == 0
        got = rb.download(np.float32, count=cnt)
        want = ((i % 100 + 1) * (n * (n + 1) // 2)).astype(np.float32)
        return np.array([np.count_nonzero(got != want)])
    if k in ("big_allreduce_rand", "big_reduce_scatter_rand"):
        # random N(0,1) fp32 at the full size, bit-exact against the oracle's simulation of the
        # algorithm the reference selects (every rank regenerates all ranks' inputs from seeds)
        from oracle import oracle
        cnt = case["count"]
        xs = [np.random.default_rng(case["seed"] * 1000 + r).standard_normal(cnt, dtype=np.float32) for r in range(n)]
        sb = m.DeviceBuffer.from_array(xs[rank])
        if k == "big_allreduce_rand":
            rb = m.DeviceBuffer(cnt * 4)
            assert L.MPI_Allreduce(sb.ptr, rb.ptr, cnt, F, OPS["MPI_SUM"], WORLD) == 0
            got = rb.download(np.uint32, count=cnt)
            want = oracle.allreduce_ref([x.view(np.uint8) for x in xs], cnt, F, OPS["MPI_SUM"])[rank].view(np.uint32)
        else:
            counts = [cnt // n + (1 if r < cnt % n else 0) for r in range(n)]
            off = sum(counts[:rank])
            rb = m.DeviceBuffer(counts[rank] * 4)
            arr = (ctypes.c_int * n)(*counts)
            assert L.MPI_Reduce_scatter(sb.ptr, rb.ptr, arr, F, OPS["MPI_SUM"], WORLD) == 0
            got = rb.download(np.uint32, count=counts[rank])
            full = oracle.reduce_scatter_ref([x.view(np.uint8) for x in xs], counts, F, OPS["MPI_SUM"]).view(np.uint32)
            want = full[off:off + counts[rank]]
        return np.array([np.count_nonzero(got != want)])
    if k == "gib_allreduce":
        # configs[2]'s upper end at any n: 1 GiB fp32 SUM.  (a) the exact pattern, every element on
        # every rank; (b) random N(0,1) operands drawn per 4 MiB block from (seed, rank, block), so
        # rank 0 can regenerate any slice of any rank: it checks a slice of `slice` floats inside
        # each ring chunk bit-exactly against the oracle's ring (oracle.allreduce algo 4 over the
        # n slices laid out as the chunks of a smaller call: chunk c keeps its rotation x_c, x_c+1 ..)
        cnt, sl = case["count"], case["slice"]
        B = 1 << 20
        per = np.resize(np.arange(1, 101, dtype=np.float32), cnt)
        sb, rb = m.DeviceBuffer.from_array(per * np.float32(rank + 1)), m.DeviceBuffer(cnt * 4)
        assert L.MPI_Allreduce(sb.ptr, rb.ptr, cnt, F, OPS["MPI_SUM"], WORLD) == 0
        bad = np.count_nonzero(rb.download(np.float32, count=cnt) != per * np.float32(n * (n + 1) // 2))
        del per

        def blocks(r, b0, nb):
            return np.concatenate([np.random.default_rng([case["seed"], r, b]).standard_normal(B, dtype=np.float32)
                                   for b in range(b0, b0 + nb)])
        sb.upload(blocks(rank, 0, cnt // B))
        assert L.MPI_Allreduce(sb.ptr, rb.ptr, cnt, F, OPS["MPI_SUM"], WORLD) == 0
        bad_rand = 0
        if rank == 0:
            from oracle import oracle
            chunk = cnt // n
            assert cnt % (n * B) == 0 and sl % B == 0 and chunk % B == 0
            offs = [c * chunk + ((c * 7 + 3) * B) % (chunk - sl + B) // B * B for c in range(n)]
            xs = [np.concatenate([blocks(r, o // B, sl // B) for o in offs]) for r in range(n)]
            want = oracle.allreduce([x.view(np.uint8) for x in xs], n * sl, F, OPS["MPI_SUM"], algo=4)[0].view(np.uint32)
            got = rb.download(np.uint32, count=cnt)
            bad_rand = sum(np.count_nonzero(got[o:o + sl] != want[c * sl:(c + 1) * sl]) for c, o in enumerate(offs))
        return np.array([bad, bad_rand])
    if k == "huge":  # operands above 4 GiB: 64-bit byte offsets through every kernel and copy
        cnt = case["count"]
        D = TYPES["MPI_DOUBLE"][0]
        i = np.arange(cnt, dtype=np.int64)
        base = (i % 1000).astype(np.float64)
        del i
        sb = m.DeviceBuffer.from_array(base * (rank + 1))
        rb = m.DeviceBuffer(cnt * 8)
        assert L.MPI_Allreduce(sb.ptr, rb.ptr, cnt, D, OPS["MPI_SUM"], WORLD) == 0  # ring wrapper + remainder
        bad_ar = np.count_nonzero(rb.download(np.float64, count=cnt) != base * (n * (n + 1) // 2))
        rb.upload(np.zeros(cnt, np.float64) if rank != 1 % n else base * (1 % n + 1))
        assert L.MPI_Bcast(rb.ptr, cnt, D, 1 % n, WORLD) == 0
        bad_bc = np.count_nonzero(rb.download(np.float64, count=cnt) != base * (1 % n + 1))
        rb.upload(base)
        assert L.MPI_Reduce_local(sb.ptr, rb.ptr, cnt, D, OPS["MPI_SUM"]) == 0
        bad_rl = np.count_nonzero(rb.download(np.float64, count=cnt) != base * (rank + 2))
        # reduce_scatter / allgather with blocks of cnt // n doubles: results past 4 GiB in total
        per = cnt // n
        counts = (ctypes.c_int * n)(*([per] * n))
        assert L.MPI_Reduce_scatter(sb.ptr, rb.ptr, counts, D, OPS["MPI_SUM"], WORLD) == 0
        want = base[rank * per:(rank + 1) * per] * (n * (n + 1) // 2)
        bad_rs = np.count_nonzero(rb.download(np.float64, count=per) != want)
        assert L.MPI_Allgather(sb.ptr, per, D, rb.ptr, per, D, WORLD) == 0
        got = rb.download(np.float64, count=per * n)
        bad_ag = sum(np.count_nonzero(got[r * per:(r + 1) * per] != base[:per] * (r + 1)) for r in range(n))
        return np.array([bad_ar, bad_bc, bad_rl, bad_rs, bad_ag])
    if k == "big_reduce_scatter":  # configs[3]: OMB recvcounts = size/n (+1 for the first size%n)
        tot = case["count"]
        counts = [tot // n + (1 if r < tot % n else 0) for r in range(n)]
        off = sum(counts[:rank])
        i = np.arange(tot, dtype=np.int64)
        x = ((i % 100 + 1) * (rank + 1)).astype(np.float32)
        sb, rb = m.DeviceBuffer.from_array(x), m.DeviceBuffer(counts[rank] * 4)
        arr = (ctypes.c_int * n)(*counts)
        assert L.MPI_Reduce_scatter(sb.ptr, rb.ptr, arr, F, OPS["MPI_SUM"], WORLD) == 0
        got = rb.download(np.float32, count=counts[rank])
        j = np.arange(off, off + counts[rank], dtype=np.int64)
        want = ((j % 100 + 1) * (n * (n + 1) // 2)).astype(np.float32)
        return np.array([np.count_nonzero(got != want)])
    if k == "big_allgather":  # configs[3]: MPI_CHAR, `per` bytes from every rank
        per = case["count"]
        C = TYPES["MPI_CHAR"][0]
        x = ((np.arange(per, dtype=np.int64) * 7 + rank) & 0xFF).astype(np.uint8)
        sb, rb = m.DeviceBuffer.from_array(x), m.DeviceBuffer(per * n)
        assert L.MPI_Allgather(sb.ptr, per, C, rb.ptr, per, C, WORLD) == 0
        got = rb.download(np.uint8, count=per * n).reshape(n, per)
        bad = 0
        for r in range(n):
            bad += np.count_nonzero(got[r] != ((np.arange(per, dtype=np.int64) * 7 + r) & 0xFF).astype(np.uint8))
        return np.array([bad])
    if k == "big_bcast":  # configs[3]: MPI_CHAR from root 0
        nbytes = case["count"]
        C = TYPES["MPI_CHAR"][0]
        want = ((np.arange(nbytes, dtype=np.int64) * 13 + 5) & 0xFF).astype(np.uint8)
        b = m.DeviceBuffer.from_array(want if rank == 0 else np.zeros(nbytes, np.uint8))
        assert L.MPI_Bcast(b.ptr, nbytes, C, 0, WORLD) == 0
        return np.array([np.count_nonzero(b.download(np.uint8, count=nbytes) != want)])
    if k == "big_maxloc":  # configs[4]: MAXLOC on MPI_DOUBLE_INT, value floor(U * 1000) (ties), loc = rank
        cnt = case["count"]
        dt = np.dtype([("value", "<f8"), ("loc", "<i4"), ("pad", "<i4")])
        vals = [np.floor(np.random.default_rng(case["seed"] * 100 + r).uniform(0, 1, cnt) * 1000) for r in range(n)]
        x = np.zeros(cnt, dt)
        x["value"], x["loc"] = vals[rank], rank
        D = TYPES["MPI_DOUBLE_INT"][0]
        sb, rb = m.DeviceBuffer.from_array(x), m.DeviceBuffer(cnt * 16)
        assert L.MPI_Allreduce(sb.ptr, rb.ptr, cnt, D, OPS["MPI_MAXLOC"], WORLD) == 0
        got = rb.download(np.uint8, count=cnt * 16).view(dt)
        v = np.stack(vals)
        mx = v.max(axis=0)
        loc = np.argmax(v == mx[None, :], axis=0)  # ties -> the lowest rank
        return np.array([np.count_nonzero((got["value"] != mx) | (got["loc"] != loc))])
    raise ValueError(k)


P = ctypes.c_void_p  # the plugin entries have no ctypes prototypes: pass pointers as pointers
_COMM = ctypes.c_void_p(0xC0FFEE0)  # stands for MVAPICH2's MPID_Comm * (opaque to the plugin)


def derived_no_alloc(L, case, rank, n):
    """Derived-type MPI_Bcast, MPI_Allgather and non-contiguous MPI_Isend / MPI_Irecv on device
    buffers: every result checked against its closed form; returns [wrong results, device
    allocations inside the calls after the warm-up round (mv2h_get_info "call_allocs"), the
    OSU-style mean latency of the derived MPI_Bcast in us]."""
    F = TYPES["MPI_FLOAT"][0]
    nb = case["nblocks"]  # MPI_Type_vector(nb, 4, 8, MPI_FLOAT): 16 * nb packed bytes
    vt = ctypes.c_int()
    assert L.MPI_Type_vector(nb, 4, 8, F, ctypes.byref(vt)) == 0
    assert L.MPI_Type_commit(ctypes.byref(vt)) == 0
    span = nb * 8
    onmap = (np.arange(span) % 8) < 4
    pat = lambda r: (np.arange(span, dtype=np.int64) * 3 + 101 * r).astype(np.float32)  # noqa: E731
    bb, ag = m.DeviceBuffer(span * 4), m.DeviceBuffer(span * 4 * n)
    sb, rb = m.DeviceBuffer.from_array(pat(rank)), m.DeviceBuffer(span * 4)
    bad = 0

    def one_round(check):
        nonlocal bad
        bb.upload(pat(0) if rank == 0 else np.full(span, -1, dtype=np.float32))
        assert L.MPI_Bcast(bb.ptr, 1, vt.value, 0, WORLD) == 0
        ag.upload(np.full(span * n, -2, dtype=np.float32))
        assert L.MPI_Allgather(sb.ptr, 1, vt.value, ag.ptr, 1, vt.value, WORLD) == 0
        rb.upload(np.full(span, -3, dtype=np.float32))
        rq = (ctypes.c_int * 2)()
        q = ctypes.c_int()
        assert L.MPI_Irecv(rb.ptr, 1, vt.value, (rank - 1) % n, 9, WORLD, ctypes.byref(q)) == 0
        rq[0] = q.value
        assert L.MPI_Isend(sb.ptr, 1, vt.value, (rank + 1) % n, 9, WORLD, ctypes.byref(q)) == 0
        rq[1] = q.value
        assert L.MPI_Waitall(2, rq, None) == 0
        if check:
            b = bb.download(np.float32, count=span)
            want = np.where(onmap, pat(0), np.float32(-1) if rank else pat(0))
            bad += int(not np.array_equal(b, want))
            # block r of the receive buffer starts r extents in (extent = span - 4 floats)
            ext = span - 4
            want = np.full(span * n, -2, dtype=np.float32)
            for r in range(n):
                want[r * ext:(r + 1) * ext] = np.where(onmap[:ext], pat(r)[:ext], np.float32(-2))
            bad += int(not np.array_equal(ag.download(np.float32, count=span * n), want))
            g = rb.download(np.float32, count=span)
            bad += int(not np.array_equal(g, np.where(onmap, pat((rank - 1) % n), np.float32(-3))))

    one_round(True)  # warm-up: grows the pooled device temporaries once
    a0 = m.info("call_allocs")
    for _ in range(case.get("rounds", 10)):
        one_round(True)
    allocs = m.info("call_allocs") - a0
    # osu_bcast.c pattern: barrier, then per iteration t0 / MPI_Bcast / t1 / barrier; mean over ranks
    iters = case.get("lat_iters", 200)
    for _ in range(20):
        L.MPI_Bcast(bb.ptr, 1, vt.value, 0, WORLD)
    L.MPI_Barrier(WORLD)
    tot = 0.0
    for _ in range(iters):
        t0 = time.perf_counter()
        L.MPI_Bcast(bb.ptr, 1, vt.value, 0, WORLD)
        tot += time.perf_counter() - t0
        L.MPI_Barrier(WORLD)
    assert L.MPI_Type_free(ctypes.byref(vt)) == 0
    return np.array([bad, allocs, tot / iters * 1e6, m.info("pool_trims")], dtype=np.float64)


def arg_checks(L, rank, n):
    """The reference's argument checks on the device path (mpierrs.h buffer tests, committed
    types, MPI_Pack's space check): every call below fails on every rank that makes it, before
    entering a collective, with the class the reference returns; then one valid MPI_Allreduce
    proves no rank was left inside a collective.  Returns [got, want] pairs per call, and the
    valid call's wrong elements last."""
    I, SUM = TYPES["MPI_INT"][0], OPS["MPI_SUM"]
    P = ctypes.c_void_p
    IN_PLACE, NULL = P(-1 & 0xFFFFFFFFFFFFFFFF), P(0)
    BUF, TYPE, COMM, ARG = 1, 3, 5, 12
    x = np.arange(4 * n, dtype=np.int32) + 10 * rank
    a, b = m.DeviceBuffer.from_array(x), m.DeviceBuffer(16 * n)
    vt, vd, vu = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert L.MPI_Type_vector(2, 1, 2, I, ctypes.byref(vt)) == 0 and L.MPI_Type_commit(ctypes.byref(vt)) == 0
    assert L.MPI_Type_dup(vt.value, ctypes.byref(vd)) == 0  # a committed type's copy is committed
    assert L.MPI_Type_vector(2, 1, 2, I, ctypes.byref(vu)) == 0  # never committed
    hip = ctypes.CDLL("libamdhip64.so")
    st = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(st)) == 0
    counts = (ctypes.c_int * n)(*([4] * n))
    req, pos = ctypes.c_int(-7), ctypes.c_int(0)
    out = m.DeviceBuffer(64)
    calls = [
        (L.MPI_Reduce_local(P(a.ptr), P(a.ptr), 4, I, SUM), BUF),  # reduce_local.c:234
        (L.MPI_Allreduce(P(a.ptr), P(a.ptr), 4, I, SUM, WORLD), BUF),  # allreduce.c:881
        (L.MPI_Allreduce(P(a.ptr), IN_PLACE, 4, I, SUM, WORLD), BUF),  # :887
        (L.MPI_Allreduce(NULL, P(b.ptr), 4, I, SUM, WORLD), BUF),  # :885
        (L.MPI_Allreduce(P(a.ptr), NULL, 4, I, SUM, WORLD), BUF),  # :888
        (L.MPI_Allreduce(P(a.ptr), P(a.ptr), 0, I, SUM, WORLD), 0),  # count 0: no alias test, no call
        # reduce.c:1194-1202: aliasing at the root; MPI_IN_PLACE is no send buffer elsewhere
        (L.MPI_Reduce(P(a.ptr), P(a.ptr), 4, I, SUM, 0, WORLD) if rank == 0 else
         L.MPI_Reduce(IN_PLACE, P(b.ptr), 4, I, SUM, 0, WORLD), BUF),
        (L.MPI_Reduce_scatter(P(a.ptr), P(a.ptr), counts, I, SUM, WORLD), BUF),  # red_scat.c:1186
        (L.MPI_Reduce_scatter_block(P(a.ptr), P(a.ptr), 4, I, SUM, WORLD), BUF),  # red_scat_block.c:1151
        (L.MPI_Reduce_scatter_block(P(a.ptr), IN_PLACE, 4, I, SUM, WORLD), BUF),  # :1147
        # allgather.c:957: the send buffer is this rank's block of the receive buffer
        (L.MPI_Allgather(P(a.ptr + 16 * rank), 4, I, P(a.ptr), 4, I, WORLD), BUF),
        (L.MPI_Allgather(P(a.ptr), 4, I, IN_PLACE, 4, I, WORLD), BUF),  # :976
        (L.MPI_Bcast(NULL, 4, I, 0, WORLD), BUF),  # bcast.c:1582
        (L.MPI_Bcast(IN_PLACE, 4, I, 0, WORLD), BUF),  # :1581
        # uncommitted derived types (MPID_Datatype_committed_ptr)
        (L.MPI_Bcast(P(b.ptr), 1, vu.value, 0, WORLD), TYPE),
        (L.MPI_Allgather(P(a.ptr), 1, vu.value, P(b.ptr), 1, vu.value, WORLD), TYPE),
        (L.MPI_Pack(P(a.ptr), 1, vu.value, P(out.ptr), 64, ctypes.byref(pos), WORLD), TYPE),  # pack.c:241
        (L.MPI_Pack(P(a.ptr), 1, vd.value, P(out.ptr), 64, ctypes.byref(pos), WORLD), 0),
        (L.MPI_Pack(P(a.ptr), 4, vt.value, P(out.ptr), 16, ctypes.byref(pos), WORLD), ARG),  # pack.c:272
        (L.MPI_Pack(P(a.ptr), 1, vt.value, P(out.ptr), 64, ctypes.byref(pos), 0x1234), COMM),
        (L.MPI_Iallreduce(P(a.ptr), P(a.ptr), 4, I, SUM, WORLD, ctypes.byref(req)), BUF),
        (req.value, -7),  # no request was made
        (L.MPIX_Allreduce_enqueue(P(a.ptr), P(a.ptr), 4, I, SUM, WORLD, st), BUF),
        (L.MPIX_Bcast_enqueue(NULL, 4, I, 0, WORLD, st), BUF),
        # MPI_COMM_SELF has no handler of its own: MPI_COMM_WORLD's (ERRORS_RETURN here) applies
        (L.MPI_Allreduce(P(a.ptr), P(a.ptr), 4, I, SUM, 0x44000001), BUF),
    ]
    assert hip.hipStreamSynchronize(st) == 0
    hip.hipStreamDestroy(st)
    for t in (vt, vd, vu):
        L.MPI_Type_free(ctypes.byref(t))
    assert L.MPI_Allreduce(P(a.ptr), P(b.ptr), 4 * n, I, SUM, WORLD) == 0
    want = sum(np.arange(4 * n, dtype=np.int32) + 10 * r for r in range(n))
    bad = int(np.count_nonzero(b.download(np.int32, count=4 * n) != want))
    return np.array([v for c in calls for v in c] + [bad], dtype=np.int64)


def soak(L, case, rank, n):
    """A long seeded sequence of small and mid-size calls back to back on the same buffers —
    blocking, nonblocking and stream-ordered collectives of every kind, one-shot and pipelined
    sizes, rotating roots, and point-to-point rings through the copy kernels — each result checked
    in place against its closed form (int32 SUM / MAX / BXOR, exact whatever the order).  The
    arenas' two slot parities, the epochs and both completion words turn over thousands of times,
    which a visibility or slot-reuse hazard that strikes once in thousands of calls would not
    survive.  Returns [wrong calls, calls made, first wrong call index or -1]."""
    I = TYPES["MPI_INT"][0]
    ops = [("MPI_SUM", OPS["MPI_SUM"]), ("MPI_MAX", OPS["MPI_MAX"]), ("MPI_BXOR", OPS["MPI_BXOR"])]
    kinds = case.get("kinds", ["allreduce", "allreduce_inplace", "iallreduce", "enqueue", "reduce",
                               "reduce_scatter_block", "allgather", "bcast", "sendrecv"])
    sizes = case.get("sizes", [1, 3, 64, 1000, 4096, 16385, 65536, 262143, 1 << 20])
    rng = np.random.default_rng(case["seed"])  # the same sequence on every rank
    mx = max(sizes)
    base = (np.arange(mx * n, dtype=np.int64) * 2654435761) % (1 << 31)
    sb, rb = m.DeviceBuffer(mx * n * 4), m.DeviceBuffer(mx * n * 4)
    hip = ctypes.CDLL("libamdhip64.so")
    st = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(st)) == 0
    P = ctypes.c_void_p
    IN_PLACE = P(-1 & 0xFFFFFFFFFFFFFFFF)
    req = ctypes.c_int()

    def pat(r, i, cnt):
        return (base[:cnt] + r * 131 + i * 7).astype(np.int32)

    def fold(op, arrs):
        out = arrs[0].astype(np.int64)
        for a in arrs[1:]:
            a = a.astype(np.int64)
            out = out + a if op == "MPI_SUM" else (np.maximum(out, a) if op == "MPI_MAX" else out ^ a)
        return out.astype(np.int32)

    wrong, first = 0, -1
    detail, ux_calls = [], 0
    sb_pre_bad, sb_post_bad, sb_detail = 0, 0, []
    calls = case["calls"]
    for i in range(calls):
        k = kinds[int(rng.integers(len(kinds)))]
        cnt = int(sizes[int(rng.integers(len(sizes)))])
        oname, op = ops[int(rng.integers(len(ops)))]
        root = int(rng.integers(n))
        if k == "reduce_scatter_block" or k == "allgather":
            cnt = max(1, cnt // n)
        mine = pat(rank, i, cnt * (n if k == "reduce_scatter_block" else 1))
        if k == "allreduce_inplace":
            rb.upload(mine)
        else:
            sb.upload(mine)
        if case.get("sync_upload"):  # diagnosis: the upload finished on the device before the call
            m.check(L.mv2h_device_synchronize(), "mv2h_device_synchronize")
        ux0 = m.info("p2p_unexpected") if case.get("detail") == 1 else 0
        if case.get("check_sb") and k == "allreduce":  # diagnosis: the operand as uploaded, before the call
            sb_pre_bad += int(not np.array_equal(sb.download(np.int32, count=cnt), mine))
        rc = 0
        if k == "allreduce":
            rc = L.MPI_Allreduce(P(sb.ptr), P(rb.ptr), cnt, I, op, WORLD)
        elif k == "allreduce_inplace":
            rc = L.MPI_Allreduce(IN_PLACE, P(rb.ptr), cnt, I, op, WORLD)
        elif k == "iallreduce":
            rc = L.MPI_Iallreduce(P(sb.ptr), P(rb.ptr), cnt, I, op, WORLD, ctypes.byref(req))
            rc = rc or L.MPI_Wait(ctypes.byref(req), None)
        elif k == "enqueue":
            rc = L.MPIX_Allreduce_enqueue(P(sb.ptr), P(rb.ptr), cnt, I, op, WORLD, st)
            rc = rc or hip.hipStreamSynchronize(st)
        elif k == "reduce":
            rc = L.MPI_Reduce(P(sb.ptr), P(rb.ptr), cnt, I, op, root, WORLD)
        elif k == "reduce_scatter_block":
            rc = L.MPI_Reduce_scatter_block(P(sb.ptr), P(rb.ptr), cnt, I, op, WORLD)
        elif k == "allgather":
            rc = L.MPI_Allgather(P(sb.ptr), cnt, I, P(rb.ptr), cnt, I, WORLD)
        elif k == "bcast":
            if rank != root:
                sb.upload(np.full(cnt, -5, dtype=np.int32))
            rc = L.MPI_Bcast(P(sb.ptr), cnt, I, root, WORLD)
        else:  # a ring of point-to-point messages
            rc = L.MPI_Sendrecv(P(sb.ptr), cnt, I, (rank + 1) % n, i % 30000, P(rb.ptr), cnt, I, (rank - 1) % n,
                                i % 30000, WORLD, None)
        if rc:
            raise RuntimeError(f"call {i} ({k}, {cnt}) returned {rc}")
        if case.get("check_sb") and k == "allreduce":  # ... and after it: a send buffer is read only
            post = sb.download(np.int32, count=cnt)
            if not np.array_equal(post, mine):
                sb_post_bad += 1
                if len(sb_detail) < 30:
                    bad = np.nonzero(post != mine)[0]
                    d = post[bad[0]].astype(np.int64) - mine[bad[0]].astype(np.int64)
                    sb_detail.extend([i, len(bad), int(bad[0]), int(bad[-1]), int(d)])
        if k in ("allreduce", "allreduce_inplace", "iallreduce", "enqueue"):
            got, want = rb.download(np.int32, count=cnt), fold(oname, [pat(r, i, cnt) for r in range(n)])
        elif k == "reduce":
            if rank != root:
                continue
            got, want = rb.download(np.int32, count=cnt), fold(oname, [pat(r, i, cnt) for r in range(n)])
        elif k == "reduce_scatter_block":
            got = rb.download(np.int32, count=cnt)
            want = fold(oname, [pat(r, i, cnt * n)[rank * cnt:(rank + 1) * cnt] for r in range(n)])
        elif k == "allgather":
            got, want = rb.download(np.int32, count=cnt * n), np.concatenate([pat(r, i, cnt) for r in range(n)])
        elif k == "bcast":
            got, want = sb.download(np.int32, count=cnt), pat(root, i, cnt)
        else:
            got, want = rb.download(np.int32, count=cnt), pat((rank - 1) % n, i, cnt)
        if not np.array_equal(got, want):
            wrong += 1
            first = i if first < 0 else first
            if case.get("detail") and len(detail) < 40:  # diagnosis: call, op, count, wrong-element span
                bad = np.nonzero(got != want)[0]
                detail.extend([i, ops.index((oname, op)), cnt, len(bad), int(bad[0]), int(bad[-1]),
                               m.info("p2p_unexpected") - ux0 if case.get("detail") == 1 else -1])
        if case.get("detail") == 1:
            ux_calls += int(m.info("p2p_unexpected") > ux0)
    hip.hipStreamDestroy(st)
    if case.get("check_sb"):
        return np.array([wrong, calls, first, sb_pre_bad, sb_post_bad] + sb_detail, dtype=np.int64)
    return np.array([wrong, calls, first] + ([ux_calls] if case.get("detail") else []) + detail, dtype=np.int64)


def collops_comm(L, rank, n):
    assert L.MV2AMD_Comm_attach(_COMM, rank, n) == 0
    return _COMM


def upload_churn(L, case, rank, n):
    """Diagnosis of the r06u / r06al / r06am stall: small blocking allreduces, with `churn_bytes` of
    freshly allocated pageable host memory uploaded (hipMemcpy) and freed between calls on the ranks
    in case["churn_ranks"] ("fresh"), or the same bytes from one array kept for the whole run
    ("kept").  Returns [first failing call or -1, calls made, wrong results]."""
    I, SUM = TYPES["MPI_INT"][0], OPS["MPI_SUM"]
    nb = case["churn_bytes"]
    scratch = m.DeviceBuffer(nb)
    kept = np.ones(nb // 4, dtype=np.int32)
    sb, rb = m.DeviceBuffer(64), m.DeviceBuffer(64)
    fail, wrong = -1, 0
    i = 0
    for i in range(case["calls"]):
        if rank in case["churn_ranks"]:
            if case["mode"] == "fresh":
                junk = np.full(nb // 4, i, dtype=np.int32)
                scratch.upload(junk)
                del junk
            else:
                kept[0] = i
                scratch.upload(kept)
        sb.upload(np.full(16, rank + i, dtype=np.int32))
        rc = L.MPI_Allreduce(P(sb.ptr), P(rb.ptr), 16, I, SUM, WORLD)
        if rc:
            fail = i
            break
        want = sum(r + i for r in range(n))
        wrong += int(not np.array_equal(rb.download(np.int32, count=16), np.full(16, want, dtype=np.int32)))
    return np.array([fail, i + 1, wrong], dtype=np.int64)


def main():
    spec = json.load(open(sys.argv[1]))
    out = sys.argv[2]
    rank = int(os.environ["RANK"])
    n = int(os.environ["WORLD_SIZE"])
    if os.environ.get("MV2AMD_TEST_HIP_FIRST") == "1":  # a host framework started HIP before the library
        nd = ctypes.c_int()
        assert ctypes.CDLL("libamdhip64.so").hipGetDeviceCount(ctypes.byref(nd)) == 0 and nd.value > 0
    L = m.lib()
    m.check(L.MPI_Init(None, None), "MPI_Init")
    L.MPI_Comm_set_errhandler(WORLD, 0x54000001)
    golden = None
    for case in spec["cases"]:
        k = case["kind"]
        t = case.get("type", "MPI_FLOAT")
        h, ext = TYPES[t][0], TYPES[t][3]
        count = case.get("count", 0)
        res = None
        if k in ("allreduce", "allreduce_inplace", "reduce", "iallreduce", "ireduce"):
            if "golden" in case:
                if golden is None:
                    golden = np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False)
                x = golden[case["golden"] + "__in"][rank]
            else:
                x = inputs(case, rank)
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(count * ext)
            rb.upload(np.full(count * ext, 0xA5, dtype=np.uint8))
            op = OPS[case["op"]]
            if case.get("via") == "collops":  # include/mv2amd_collops.h (MPID_Collops entries)
                comm, err = collops_comm(L, rank, n), ctypes.c_int(0)
                if k == "allreduce":
                    rc = L.MV2AMD_Allreduce(P(sb.ptr), P(rb.ptr), count, h, op, comm, ctypes.byref(err))
                else:
                    rc = L.MV2AMD_Reduce(P(sb.ptr), P(rb.ptr), count, h, op, case["root"], comm, ctypes.byref(err))
                assert err.value == 0
            elif k == "allreduce":
                rc = L.MPI_Allreduce(sb.ptr, rb.ptr, count, h, op, WORLD)
            elif k == "allreduce_inplace":
                rc = L.MPI_Allreduce(ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF), sb.ptr, count, h, op, WORLD)
                rb = sb
            elif k == "iallreduce":  # nonblocking: initiate, then MPI_Wait (completion word)
                req = ctypes.c_int()
                rc = L.MPI_Iallreduce(sb.ptr, rb.ptr, count, h, op, WORLD, ctypes.byref(req))
                if rc == 0:
                    rc = L.MPI_Wait(ctypes.byref(req), None)
            elif k == "ireduce":
                req = ctypes.c_int()
                rc = L.MPI_Ireduce(sb.ptr, rb.ptr, count, h, op, case["root"], WORLD, ctypes.byref(req))
                if rc == 0:
                    rc = L.MPI_Wait(ctypes.byref(req), None)
            else:
                rc = L.MPI_Reduce(sb.ptr, rb.ptr, count, h, op, case["root"], WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=count * ext)
        elif k == "graph_allreduce":  # HIP graph capture of MPIX_Allreduce_enqueue (graph lane)
            res = graph_allreduce(L, case, rank, n)
        elif k == "graph_collectives":  # every stream-ordered collective in one captured graph
            res = graph_collectives(L, case, rank, n)
        elif k == "enqueue_seq":  # stream-ordered collectives (MPIX_*_enqueue) mixed with a blocking call
            res = enqueue_seq(L, case, rank, n)
        elif k == "tiling_info":  # pipelined kernels' tiling after MPI_Init (pipe_autotune)
            keys = ["pipe_tuned", "pipe_grid", "pipe_sub", "tune_n", "pipe_rnt", "oneshot_max", "os_tune_n",
                    "selftest_calls", "hw_queues_set", "code_load_us"]
            res = np.array([m.info(key) for key in keys], dtype=np.int64)
        elif k == "mpit_counts":  # MPI_T: start every counter, run the calls, read the counters
            prov = ctypes.c_int()
            assert L.MPI_T_init_thread(3, ctypes.byref(prov)) == 0
            sess, npv = ctypes.c_void_p(), ctypes.c_int()
            assert L.MPI_T_pvar_session_create(ctypes.byref(sess)) == 0
            assert L.MPI_T_pvar_get_num(ctypes.byref(npv)) == 0
            names, handles = [], []
            for i in range(npv.value):
                nm, nl, cls = ctypes.create_string_buffer(128), ctypes.c_int(128), ctypes.c_int()
                assert L.MPI_T_pvar_get_info(i, nm, ctypes.byref(nl), None, ctypes.byref(cls), None, None, None, None,
                                             None, None, None, None) == 0
                if cls.value != 246:  # counters only
                    continue
                hd, cnt = ctypes.c_void_p(), ctypes.c_int()
                assert L.MPI_T_pvar_handle_alloc(sess, i, None, ctypes.byref(hd), ctypes.byref(cnt)) == 0
                names.append(nm.value.decode())
                handles.append(hd)
            assert L.MPI_T_pvar_start(sess, ctypes.c_void_p.in_dll(L, "MPI_T_PVAR_ALL_HANDLES")) == 0
            for call in case["calls"]:
                cnt, tt = call["count"], TYPES[call["type"]][0]
                e = TYPES[call["type"]][3]
                sb, rb = m.DeviceBuffer(max(16, cnt * e * n)), m.DeviceBuffer(max(16, cnt * e * n))
                if call["coll"] == "allreduce":
                    src = ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF) if call.get("in_place") else sb.ptr
                    rc = L.MPI_Allreduce(src, rb.ptr, cnt, tt, OPS["MPI_SUM"], WORLD)
                elif call["coll"] == "reduce":
                    rc = L.MPI_Reduce(sb.ptr, rb.ptr, cnt, tt, OPS["MPI_SUM"], call["root"], WORLD)
                else:
                    rc = L.MPI_Reduce_scatter(sb.ptr, rb.ptr, (ctypes.c_int * n)(*([cnt] * n)), tt, OPS["MPI_SUM"],
                                              WORLD)
                assert rc == 0, (call, rc)
            assert L.MPI_T_pvar_stop(sess, ctypes.c_void_p.in_dll(L, "MPI_T_PVAR_ALL_HANDLES")) == 0
            vals = {}
            for nm, hd in zip(names, handles):
                v = ctypes.c_ulonglong()
                assert L.MPI_T_pvar_read(sess, hd, ctypes.byref(v)) == 0
                vals[nm] = v.value
            assert L.MPI_T_pvar_session_free(ctypes.byref(sess)) == 0
            assert L.MPI_T_finalize() == 0
            res = np.frombuffer(json.dumps(vals).encode(), dtype=np.uint8)
        elif k == "reduce_scatter":
            counts = case["recvcounts"]
            x = inputs(dict(case, count=sum(counts)), rank)
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(max(1, counts[rank]) * ext)
            arr = (ctypes.c_int * n)(*counts)
            if case.get("via") == "collops":
                rc = L.MV2AMD_Reduce_scatter(P(sb.ptr), P(rb.ptr), arr, h, OPS[case["op"]], collops_comm(L, rank, n), None)
            elif case.get("via") in ("block", "iblock", "inb"):
                req = ctypes.c_int()
                if case["via"] == "block":
                    rc = L.MPI_Reduce_scatter_block(P(sb.ptr), P(rb.ptr), counts[0], h, OPS[case["op"]], WORLD)
                elif case["via"] == "iblock":
                    rc = L.MPI_Ireduce_scatter_block(P(sb.ptr), P(rb.ptr), counts[0], h, OPS[case["op"]], WORLD,
                                                     ctypes.byref(req))
                else:
                    rc = L.MPI_Ireduce_scatter(P(sb.ptr), P(rb.ptr), arr, h, OPS[case["op"]], WORLD, ctypes.byref(req))
                if rc == 0 and case["via"] != "block":
                    rc = L.MPI_Wait(ctypes.byref(req), None)
            else:
                rc = L.MPI_Reduce_scatter(sb.ptr, rb.ptr, arr, h, OPS[case["op"]], WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=counts[rank] * ext)
        elif k == "allgather":
            x = inputs(case, rank)
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(count * ext * n)
            if case.get("via") == "collops":
                rc = L.MV2AMD_Allgather(P(sb.ptr), count, h, P(rb.ptr), count, h, collops_comm(L, rank, n), None)
            else:
                rc = L.MPI_Allgather(sb.ptr, count, h, rb.ptr, count, h, WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=count * ext * n)
        elif k == "bcast":
            x = inputs(case, rank)
            b = m.DeviceBuffer.from_array(x)
            if case.get("via") == "collops":
                rc = L.MV2AMD_Bcast(P(b.ptr), count, h, case["root"], collops_comm(L, rank, n), None)
            else:
                rc = L.MPI_Bcast(b.ptr, count, h, case["root"], WORLD)
            assert rc == 0, (case["id"], rc)
            res = b.download(np.uint8, count=count * ext)
        elif k == "user_allreduce":
            FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_int))

            def uop(inp, io, ln, dt):
                c = ln[0]
                a = np.ctypeslib.as_array((ctypes.c_int * c).from_address(inp))
                b = np.ctypeslib.as_array((ctypes.c_int * c).from_address(io))
                b[:] = a * 2 + b * 3
            cb = FN(uop)
            op = ctypes.c_int()
            L.MPI_Op_create(ctypes.cast(cb, ctypes.c_void_p), case["commute"], ctypes.byref(op))
            x = (np.arange(count, dtype=np.int32) + rank) % 7
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(count * 4)
            rc = L.MPI_Allreduce(sb.ptr, rb.ptr, count, TYPES["MPI_INT"][0], op.value, WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=count * 4)
            L.MPI_Op_free(ctypes.byref(op))
        elif k == "user_reduce":
            FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_int))

            def uop(inp, io, ln, dt):
                c = ln[0]
                a = np.ctypeslib.as_array((ctypes.c_int * c).from_address(inp))
                b = np.ctypeslib.as_array((ctypes.c_int * c).from_address(io))
                b[:] = a * 2 + b * 3
            cb = FN(uop)
            op = ctypes.c_int()
            L.MPI_Op_create(ctypes.cast(cb, ctypes.c_void_p), case["commute"], ctypes.byref(op))
            x = (np.arange(count, dtype=np.int32) + rank) % 7
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(count * 4)
            rc = L.MPI_Reduce(sb.ptr, rb.ptr, count, TYPES["MPI_INT"][0], op.value, case["root"], WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=count * 4)
            L.MPI_Op_free(ctypes.byref(op))
        elif k == "user_reduce_scatter":
            FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_int))

            def uop(inp, io, ln, dt):
                c = ln[0]
                a = np.ctypeslib.as_array((ctypes.c_int * c).from_address(inp))
                b = np.ctypeslib.as_array((ctypes.c_int * c).from_address(io))
                b[:] = a * 2 + b * 3
            cb = FN(uop)
            op = ctypes.c_int()
            L.MPI_Op_create(ctypes.cast(cb, ctypes.c_void_p), case["commute"], ctypes.byref(op))
            counts = case["recvcounts"]
            x = ((np.arange(sum(counts)) + rank) % 7).astype(np.int32)
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(max(1, counts[rank]) * 4)
            arr = (ctypes.c_int * n)(*counts)
            via, req, H = case.get("via"), ctypes.c_int(), TYPES["MPI_INT"][0]
            if via == "block":
                rc = L.MPI_Reduce_scatter_block(P(sb.ptr), P(rb.ptr), counts[0], H, op.value, WORLD)
            elif via == "iblock":
                rc = L.MPI_Ireduce_scatter_block(P(sb.ptr), P(rb.ptr), counts[0], H, op.value, WORLD,
                                                 ctypes.byref(req))
            elif via == "inb":
                rc = L.MPI_Ireduce_scatter(P(sb.ptr), P(rb.ptr), arr, H, op.value, WORLD, ctypes.byref(req))
            else:
                rc = L.MPI_Reduce_scatter(sb.ptr, rb.ptr, arr, H, op.value, WORLD)
            if rc == 0 and via in ("iblock", "inb"):
                rc = L.MPI_Wait(ctypes.byref(req), None)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=counts[rank] * 4)
            L.MPI_Op_free(ctypes.byref(op))
        elif k == "user_vector_allreduce":
            # configs[4]: commutative user op on MPI_Type_vector(nb, 4, 8, MPI_FLOAT) operands;
            # fn(in, io) = 0.5 in + 1.5 io on the type map only; gap bytes must stay untouched
            nb, cnt = case["nblocks"], count
            vt = ctypes.c_int()
            assert L.MPI_Type_vector(nb, 4, 8, TYPES["MPI_FLOAT"][0], ctypes.byref(vt)) == 0
            assert L.MPI_Type_commit(ctypes.byref(vt)) == 0
            ext_f = (nb - 1) * 8 + 4
            FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_int))

            def uop(inp, io, ln, dt):  # strided views of the c elements' type maps
                c = ln[0]
                shape, strides = (c, nb, 4), (ext_f * 4, 32, 4)
                a = np.lib.stride_tricks.as_strided(
                    np.ctypeslib.as_array((ctypes.c_float * (c * ext_f)).from_address(inp)), shape, strides)
                b = np.lib.stride_tricks.as_strided(
                    np.ctypeslib.as_array((ctypes.c_float * (c * ext_f)).from_address(io)), shape, strides)
                b[...] = a * np.float32(0.5) + b * np.float32(1.5)
            cb = FN(uop)
            op = ctypes.c_int()
            L.MPI_Op_create(ctypes.cast(cb, ctypes.c_void_p), 1, ctypes.byref(op))
            x = np.random.default_rng(case["seed"] * 1000 + rank).standard_normal(cnt * ext_f).astype(np.float32)
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer.from_array(np.full(cnt * ext_f, -7.0, dtype=np.float32))
            rc = L.MPI_Allreduce(sb.ptr, rb.ptr, cnt, vt.value, op.value, WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=cnt * ext_f * 4)
            # the operand bytes this rank received, and its receive area (mpi/user_coll.cpp staging)
            np.save(os.path.join(out, f"{case['id']}_staged_r{rank}.npy"),
                    np.array([m.info("uop_in_bytes"), m.info("uop_area_bytes")], dtype=np.int64))
            L.MPI_Op_free(ctypes.byref(op))
            L.MPI_Type_free(ctypes.byref(vt))
        elif k.startswith("big_") or k in ("huge", "gib_allreduce"):
            res = big_case(L, case, rank, n)
        elif k == "derived_no_alloc":
            res = derived_no_alloc(L, case, rank, n)
        elif k == "arg_checks":
            res = arg_checks(L, rank, n)
        elif k == "soak":
            res = soak(L, case, rank, n)
        elif k == "upload_churn":  # diagnosis (tools/runs/run_r06an.sh): pageable uploads between calls
            res = upload_churn(L, case, rank, n)
        elif k == "peer_absent":  # a collective one rank never enters: the others' device wait runs out
            if rank == case["absent"]:
                # into MPI_Finalize's host barrier (bounded by the same timeout) only after the peer's
                # device wait has run out and been reported
                time.sleep(case["sleep"])
                res = np.array([0], dtype=np.int64)
            else:
                sb, rb = m.DeviceBuffer.from_array(np.ones(2, dtype=np.float32)), m.DeviceBuffer(8)
                rc = L.MPI_Allreduce(sb.ptr, rb.ptr, 2, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"], WORLD)
                res = np.array([rc], dtype=np.int64)
        elif k == "vector_bcast":
            # MPI_Type_vector(N, 4, 8, MPI_FLOAT) operand broadcast (device pack/unpack path)
            vt = ctypes.c_int()
            nb = case["nblocks"]
            assert L.MPI_Type_vector(nb, 4, 8, TYPES["MPI_FLOAT"][0], ctypes.byref(vt)) == 0
            assert L.MPI_Type_commit(ctypes.byref(vt)) == 0
            x = np.full(nb * 8, -1.0, dtype=np.float32)
            if rank == case["root"]:
                x = np.arange(nb * 8, dtype=np.float32)
            b = m.DeviceBuffer.from_array(x)
            rc = L.MPI_Bcast(b.ptr, 1, vt.value, case["root"], WORLD)
            assert rc == 0, (case["id"], rc)
            res = b.download(np.uint8, count=nb * 8 * 4)
            L.MPI_Type_free(ctypes.byref(vt))
        else:
            raise ValueError(k)
        np.save(os.path.join(out, f"{case['id']}_r{rank}.npy"), res)
    L.MPI_Finalize()
    print(f"rank {rank} done", flush=True)


if __name__ == "__main__":
    main()
