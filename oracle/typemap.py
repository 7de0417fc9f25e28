"""Type-map oracle for derived datatypes (TEST INFRASTRUCTURE ONLY).

A pure-Python restatement of MPI-3.1 §4.1 type maps as the reference
builds them, independent of the product's segment flattening:

* a type is its full type map — one (displacement, basic size) entry per
  basic element, in type-map order — plus lb, ub, alignsize and size;
* constructors follow the reference's MPID_Type_* files:
  contiguous (mpid_type_contiguous.c), vector / hvector (mpid_type_vector.c),
  indexed / hindexed (mpid_type_indexed.c: blocks of length 0 are skipped for
  lb/ub, :155-200), blockindexed (mpid_type_blockindexed.c), struct
  (mpid_type_struct.c: lb/ub over non-empty blocks :215-380, alignsize
  :42-124, extent padded to alignsize :400-411), resized
  (mpid_type_create_resized.c), subarray (type_create_subarray.c: vectors +
  resized to lb 0, extent prod(sizes)·extent(old));
* pack = the bytes of every type-map entry in order, element after element
  `extent` bytes apart (Segment_pack, segment_packunpack.c:70 driving the
  m2m callbacks); unpack is its inverse and never touches other bytes.

Only tests/ use this module, as the checker.
"""
import numpy as np

FP = {0x4c00040a, 0x4c00080b, 0x4c00100c}
PAIRS = {  # handle: (entries [(disp, size)], extent, align)
    0x8c000000: ([(0, 4), (4, 4)], 8, 4),      # FLOAT_INT
    0x8c000001: ([(0, 8), (8, 4)], 16, 8),     # DOUBLE_INT
    0x8c000002: ([(0, 8), (8, 4)], 16, 8),     # LONG_INT
    0x8c000003: ([(0, 2), (4, 4)], 8, 4),      # SHORT_INT
    0x4c000816: ([(0, 4), (4, 4)], 8, 4),      # 2INT
}


class T:
    """A datatype as its type map."""

    def __init__(self, entries, lb, ub, align):
        self.entries = list(entries)  # [(disp, nbytes)]
        self.lb, self.ub, self.align = lb, ub, align

    @property
    def extent(self):
        return self.ub - self.lb

    @property
    def size(self):
        return sum(n for _, n in self.entries)

    @property
    def true_lb(self):
        return min((d for d, _ in self.entries), default=0)

    @property
    def true_extent(self):
        if not self.entries:
            return 0
        return max(d + n for d, n in self.entries) - self.true_lb


def builtin(handle):
    if handle in PAIRS:
        ent, ext, al = PAIRS[handle]
        return T(ent, 0, ext, al)
    size = (handle >> 8) & 0xFF
    align = size if handle in FP else min(size, 8)
    return T([(0, size)], 0, size, align)


def _blocks(blocks, pad=False):
    """blocks: [(disp_bytes, blocklen, T)] -> T (struct semantics)."""
    entries, lb, ub, align = [], None, None, 1
    for disp, bl, old in blocks:
        align = max(align, old.align)
        if bl == 0:
            continue
        for k in range(bl):
            base = disp + k * old.extent
            entries.extend((base + d, n) for d, n in old.entries)
        b0 = disp + old.lb
        b1 = disp + old.lb + bl * old.extent
        lo, hi = min(b0, b1), max(b0, b1)
        lb = lo if lb is None else min(lb, lo)
        ub = hi if ub is None else max(ub, hi)
    if lb is None:
        lb = ub = 0
    t = T(entries, lb, ub, align)
    if pad and align > 1 and t.extent % align:
        t.ub += align - t.extent % align
    return t


def contiguous(count, old):
    return _blocks([(i * old.extent, 1, old) for i in range(count)])


def hvector(count, blocklen, stride_bytes, old):
    return _blocks([(i * stride_bytes, blocklen, old) for i in range(count)])


def vector(count, blocklen, stride, old):
    return hvector(count, blocklen, stride * old.extent, old)


def indexed(blocklens, displs, old):
    return _blocks([(d * old.extent, b, old) for b, d in zip(blocklens, displs)])


def hindexed(blocklens, displs_bytes, old):
    return _blocks([(d, b, old) for b, d in zip(blocklens, displs_bytes)])


def indexed_block(blocklen, displs, old):
    return indexed([blocklen] * len(displs), displs, old)


def struct(blocklens, displs_bytes, types):
    return _blocks(list(zip(displs_bytes, blocklens, types)), pad=True)


def resized(old, lb, extent):
    return T(old.entries, lb, lb + extent, old.align)


def subarray(sizes, subsizes, starts, order_c, old):
    nd = len(sizes)
    dims = list(range(nd)) if order_c else list(range(nd))[::-1]  # slowest ... fastest
    strides, tot = [0] * nd, 1
    for i in range(nd - 1, -1, -1):
        strides[i] = tot
        tot *= sizes[dims[i]]
    blocks = []
    idx = np.indices([subsizes[dims[i]] for i in range(nd - 1)]).reshape(nd - 1, -1).T if nd > 1 else [()]
    for row in idx:
        e = starts[dims[-1]]
        for i, v in enumerate(row):
            e += (starts[dims[i]] + int(v)) * strides[i]
        blocks.append((e * old.extent, subsizes[dims[-1]], old))
    t = _blocks(blocks)
    return T(t.entries, 0, tot * old.extent, old.align)


def byte_index(t, count):
    """Byte offsets (relative to the buffer pointer) of the packed stream."""
    one = np.concatenate([np.arange(d, d + n, dtype=np.int64) for d, n in t.entries]) if t.entries else \
        np.zeros(0, np.int64)
    return (np.arange(count, dtype=np.int64)[:, None] * t.extent + one[None, :]).ravel()


def pack(buf, t, count):
    return buf[byte_index(t, count)].copy()


def unpack(packed, canvas, t, count):
    out = canvas.copy()
    out[byte_index(t, count)] = packed
    return out
