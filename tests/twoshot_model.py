"""Host model of the two-shot device allreduce (k_twoshot, csrc/coll/kernels_impl.h)
used by the CPU tests: tile ownership (tile t -> rank t % n), per-element
reduction order (LINEAR / BUTTERFLY with reduce-scatter owner bitrev(block)),
and the all-gather of the owners' tiles.  Arithmetic is delegated to the
oracle's op loop, so the model checks the *decomposition*, not the ops."""
import numpy as np

from oracle import oracle

TV_BYTES = 256 * 2 * 16  # kThreads * U * sizeof(v4u)


def tree_params(n, count, size):
    pof2 = 1
    while pof2 * 2 <= n:
        pof2 *= 2
    lg = pof2.bit_length() - 1
    return {"pof2": pof2, "rem": n - pof2, "lg": lg, "linear": count * size < 1024,
            "rs_blk": count // pof2 if count >= pof2 else 0}


def bitrev(b, lg):
    return int(format(b, f"0{lg}b")[::-1], 2) if lg else 0


def reduce_range(xs, e0, e1, ext, h, oh, tp, owner_fixed=None):
    """Reduce elements [e0, e1) of the n byte-buffers in `xs` in reference order."""
    n = len(xs)
    seg = [x[e0 * ext:e1 * ext].copy() for x in xs]
    cnt = e1 - e0
    if cnt == 0:
        return np.zeros(0, dtype=np.uint8)

    def ap(a, b):  # op(a, b), a = inout
        r = a.copy()
        assert oracle.reduce_local(b, r, len(r) // ext, h, oh) == 0
        return r

    if tp["linear"]:
        acc = seg[0]
        for i in range(1, n):
            acc = ap(acc, seg[i])
        return acc
    out = np.zeros(cnt * ext, dtype=np.uint8)
    # split the range by reduce-scatter block so each piece has one owner
    pieces = []
    if owner_fixed is not None:
        pieces = [(e0, e1, owner_fixed)]
    else:
        e = e0
        while e < e1:
            b = min(e // tp["rs_blk"], tp["pof2"] - 1)
            end = e1 if b == tp["pof2"] - 1 else min(e1, (b + 1) * tp["rs_blk"])
            pieces.append((e, end, bitrev(b, tp["lg"])))
            e = end
    for (a0, a1, o) in pieces:
        v = [s[(a0 - e0) * ext:(a1 - e0) * ext] for s in seg]
        w = [ap(v[2 * i + 1], v[2 * i]) if i < tp["rem"] else v[i + tp["rem"]] for i in range(tp["pof2"])]
        m = 1
        while m < tp["pof2"]:
            for j in range(0, tp["pof2"], 2 * m):
                x, y = (w[j + m], w[j]) if (o & m) else (w[j], w[j + m])
                w[j] = ap(x, y)
            m <<= 1
        out[(a0 - e0) * ext:(a1 - e0) * ext] = w[0]
    return out


def rs_tiles(xs, rank, count, ext, h, oh, tp):
    """Rank `rank`'s reduce-scatter phase: {tile index: reduced bytes} for tiles t % n == rank
    (whole 16-byte vectors only; the scalar tail is handled separately)."""
    n = len(xs)
    nvec = count * ext // 16
    tv = TV_BYTES // 16
    ntiles = (nvec + tv - 1) // tv
    out = {}
    for t in range(rank, ntiles, n):
        v0, v1 = t * tv, min((t + 1) * tv, nvec)
        e0, e1 = v0 * 16 // ext, v1 * 16 // ext
        out[t] = reduce_range(xs, e0, e1, ext, h, oh, tp)
    return out


def tail(xs, count, ext, h, oh, tp):
    nvec = count * ext // 16
    e0 = nvec * 16 // ext
    return e0, reduce_range(xs, e0, count, ext, h, oh, tp)


def assemble(tile_maps, count, ext, tail_part):
    res = np.zeros(count * ext, dtype=np.uint8)
    tv = TV_BYTES // 16
    for mp in tile_maps:
        for t, data in mp.items():
            res[t * tv * 16:t * tv * 16 + len(data)] = data
    e0, tb = tail_part
    res[e0 * ext:] = tb
    return res
