"""Host model of the pipelined push collectives (k_pipe, csrc/coll/pipe.h and
the geometry in csrc/runtime/coll.cpp): segment layout, round / workgroup
ranges, arena slots [parity][source], and the per-element reduction order
(LINEAR / BUTTERFLY with reduce-scatter owner bitrev(block)).  Arithmetic is
delegated to the oracle's op loop, so the model checks the decomposition and
data movement, not the ops."""
import numpy as np

from oracle import oracle

PIPE_MAX_GRID = 256
PIPE_MAX_SUB = 128 << 10
PIPE_SLOT = PIPE_MAX_GRID * PIPE_MAX_SUB  # bytes of one arena slot (kPipeSlot)
PIPE_MIN_SUB = 16 << 10


def pipe_geom(maxlen, cus=256, nshare=1, pipe_grid=PIPE_MAX_GRID, pipe_sub=PIPE_MAX_SUB):
    """coll.cpp pipe_geom(): (grid, tsub, tseg, nrounds)."""
    cap = min(PIPE_MAX_GRID, max(1, cus // max(1, nshare)), max(1, pipe_grid))
    g = min(cap, max(1, -(-maxlen // PIPE_MIN_SUB)))
    tsub = -(-maxlen // g)
    tsub = (tsub + 4095) & ~4095
    tsub = min(tsub, min(PIPE_SLOT // g, max(4096, pipe_sub)) & ~4095)
    tseg = g * tsub
    return g, tsub, tseg, -(-maxlen // tseg)


def even_segments(nbytes, n):
    """coll.cpp even_segments(): [(offset, length)] per rank, 16-byte aligned."""
    seg = ((-(-nbytes // n)) + 15) & ~15
    out = []
    for j in range(n):
        off = min(j * seg, nbytes)
        out.append((off, min(seg, nbytes - off)))
    return out


def tree_params(n, count, size):
    pof2 = 1
    while pof2 * 2 <= n:
        pof2 *= 2
    lg = pof2.bit_length() - 1
    return {"pof2": pof2, "rem": n - pof2, "lg": lg, "linear": count * size <= 1024,
            "rs_blk": count // pof2 if count >= pof2 else 0}


def ring_segments(count, ext, n):
    """coll.cpp AR_RING: segment j = ring chunk j of count/n elements (count % n == 0)."""
    cb = (count // n) * ext
    return [(j * cb, cb) for j in range(n)]


def bitrev(b, lg):
    return int(format(b, f"0{lg}b")[::-1], 2) if lg else 0


def _ap(a, b, ext, h, oh):  # op(a, b), a = inout
    r = a.copy()
    assert oracle.reduce_local(b, r, len(r) // ext, h, oh) == 0
    return r


def reduce_range(seg, e0, ext, h, oh, tp):
    """Reduce the n byte-arrays `seg` (elements [e0, e0+len)) in reference order."""
    n = len(seg)
    cnt = len(seg[0]) // ext
    if cnt == 0:
        return np.zeros(0, dtype=np.uint8)
    if tp.get("ring") is not None:
        # flat ring allreduce: chunk `ring` starts at rank ring, the partial is the accumulator
        r0 = tp["ring"]
        acc = seg[r0]
        for k in range(1, n):
            acc = _ap(acc, seg[(r0 + k) % n], ext, h, oh)
        return acc
    if tp["linear"]:
        acc = seg[0]
        for i in range(1, n):
            acc = _ap(acc, seg[i], ext, h, oh)
        return acc
    out = np.zeros(cnt * ext, dtype=np.uint8)
    e, e1 = e0, e0 + cnt
    while e < e1:
        b = min(e // tp["rs_blk"], tp["pof2"] - 1)
        end = e1 if b == tp["pof2"] - 1 else min(e1, (b + 1) * tp["rs_blk"])
        o = bitrev(b, tp["lg"])
        v = [s[(e - e0) * ext:(end - e0) * ext] for s in seg]
        rem = tp["rem"]
        w = [_ap(v[2 * i + 1], v[2 * i], ext, h, oh) if i < rem else v[i + rem] for i in range(tp["pof2"])]
        m = 1
        while m < tp["pof2"]:
            for j in range(0, tp["pof2"], 2 * m):
                x, y = (w[j + m], w[j]) if (o & m) else (w[j], w[j + m])
                w[j] = _ap(x, y, ext, h, oh)
            m <<= 1
        out[(e - e0) * ext:(end - e0) * ext] = w[0]
        e = end
    return out


def allreduce(xs, count, ext, h, oh, tp, geom_kw=None):
    """Simulate PIPE_AR on n ranks: every byte crosses 'GPUs' only through the
    arena slots.  Returns the n recv buffers."""
    n = len(xs)
    nbytes = count * ext
    ring = tp.get("ring_mode", False)
    segs = ring_segments(count, ext, n) if ring else even_segments(nbytes, n)
    g, tsub, tseg, nrounds = pipe_geom(max(l for _, l in segs), **(geom_kw or {}))
    rs = [{} for _ in range(n)]  # rs[dst][(par, src)] -> bytearray slot
    ag = [{} for _ in range(n)]
    recv = [np.zeros(nbytes, dtype=np.uint8) for _ in range(n)]

    def slot(region, dst, par, src):
        return region[dst].setdefault((par, src), np.zeros(tseg, dtype=np.uint8))

    for k in range(nrounds):
        par = k & 1
        for b in range(g):
            rbase, soff = k * tseg + b * tsub, b * tsub

            def rng(j):
                off, ln = segs[j]
                return (off + rbase, min(tsub, ln - rbase)) if rbase < ln else (0, 0)
            for p in range(n):          # P1 scatter
                for j in range(n):
                    if j != p:
                        o, ln = rng(j)
                        if ln:
                            slot(rs, j, par, p)[soff:soff + ln] = xs[p][o:o + ln]
            for r in range(n):          # P2 reduce own segment, push
                o, ln = rng(r)
                if not ln:
                    continue
                ops = [xs[r][o:o + ln] if j == r else slot(rs, r, par, j)[soff:soff + ln] for j in range(n)]
                res = reduce_range(ops, o // ext, ext, h, oh, dict(tp, ring=r) if ring else tp)
                recv[r][o:o + ln] = res
                for j in range(n):
                    if j != r:
                        slot(ag, j, par, r)[soff:soff + ln] = res
            for r in range(n):          # P3 gather
                for j in range(n):
                    o, ln = rng(j)
                    if j != r and ln:
                        recv[r][o:o + ln] = slot(ag, r, par, j)[soff:soff + ln]
    return recv
