"""Derived-datatype cases built twice: through the library's MPI_Type_*
constructors and through the type-map oracle (oracle/typemap.py).

The shapes restate the reference's datatype tests: simple-pack.c (vector of
int), pairtype-pack.c / pairtype-size-extent.c (pair types, struct padding),
slice-pack.c (vector of vector), vecblklen.c, zero-blklen-vector.c (blocks
of length 0), indexed / struct / subarray / resized combinations, plus the
BASELINE config-5 operand MPI_Type_vector(N, 4, 8, MPI_FLOAT)."""
import ctypes

from oracle import typemap as tm

FLOAT, DOUBLE, INT, CHAR, SHORT = 0x4c00040a, 0x4c00080b, 0x4c000405, 0x4c000101, 0x4c000203
DOUBLE_INT, SHORT_INT, LONG_INT = 0x8c000001, 0x8c000003, 0x8c000002


def _ia(v):
    return (ctypes.c_int * max(1, len(v)))(*v)


def _la(v):
    return (ctypes.c_long * max(1, len(v)))(*v)


class Built:
    """(library handle, oracle type) pair; frees the library handles on close."""

    def __init__(self, L):
        self.L = L
        self.handles = []

    def _new(self, rc, h):
        assert rc == 0, rc
        self.handles.append(h)
        return h.value

    def lib_type(self, spec):
        """spec: nested tuples, e.g. ("vector", 3, 2, 4, ("builtin", FLOAT))."""
        kind = spec[0]
        L = self.L
        if kind == "builtin":
            return spec[1]
        h = ctypes.c_int()
        if kind == "contiguous":
            return self._new(L.MPI_Type_contiguous(spec[1], self.lib_type(spec[2]), ctypes.byref(h)), h)
        if kind == "vector":
            return self._new(L.MPI_Type_vector(spec[1], spec[2], spec[3], self.lib_type(spec[4]), ctypes.byref(h)), h)
        if kind == "hvector":
            return self._new(L.MPI_Type_create_hvector(spec[1], spec[2], spec[3], self.lib_type(spec[4]),
                                                       ctypes.byref(h)), h)
        if kind == "indexed":
            bl, ds = spec[1], spec[2]
            return self._new(L.MPI_Type_indexed(len(bl), _ia(bl), _ia(ds), self.lib_type(spec[3]), ctypes.byref(h)), h)
        if kind == "hindexed":
            bl, ds = spec[1], spec[2]
            return self._new(L.MPI_Type_create_hindexed(len(bl), _ia(bl), _la(ds), self.lib_type(spec[3]),
                                                        ctypes.byref(h)), h)
        if kind == "indexed_block":
            ds = spec[2]
            return self._new(L.MPI_Type_create_indexed_block(len(ds), spec[1], _ia(ds), self.lib_type(spec[3]),
                                                             ctypes.byref(h)), h)
        if kind == "hindexed_block":
            ds = spec[2]
            return self._new(L.MPI_Type_create_hindexed_block(len(ds), spec[1], _la(ds), self.lib_type(spec[3]),
                                                              ctypes.byref(h)), h)
        if kind == "struct":
            bl, ds, ts = spec[1], spec[2], [self.lib_type(t) for t in spec[3]]
            return self._new(L.MPI_Type_create_struct(len(bl), _ia(bl), _la(ds), _ia(ts), ctypes.byref(h)), h)
        if kind == "resized":
            return self._new(L.MPI_Type_create_resized(self.lib_type(spec[1]), spec[2], spec[3], ctypes.byref(h)), h)
        if kind == "dup":
            return self._new(L.MPI_Type_dup(self.lib_type(spec[1]), ctypes.byref(h)), h)
        if kind == "subarray":
            sz, sub, st, order = spec[1], spec[2], spec[3], spec[4]
            return self._new(L.MPI_Type_create_subarray(len(sz), _ia(sz), _ia(sub), _ia(st), order,
                                                        self.lib_type(spec[5]), ctypes.byref(h)), h)
        raise ValueError(kind)

    def close(self):
        for h in self.handles:
            self.L.MPI_Type_free(ctypes.byref(h))
        self.handles = []


def oracle_type(spec):
    kind = spec[0]
    if kind == "builtin":
        return tm.builtin(spec[1])
    if kind == "contiguous":
        return tm.contiguous(spec[1], oracle_type(spec[2]))
    if kind == "vector":
        return tm.vector(spec[1], spec[2], spec[3], oracle_type(spec[4]))
    if kind == "hvector":
        return tm.hvector(spec[1], spec[2], spec[3], oracle_type(spec[4]))
    if kind == "indexed":
        return tm.indexed(spec[1], spec[2], oracle_type(spec[3]))
    if kind == "hindexed":
        return tm.hindexed(spec[1], spec[2], oracle_type(spec[3]))
    if kind == "indexed_block":
        return tm.indexed_block(spec[1], spec[2], oracle_type(spec[3]))
    if kind == "hindexed_block":
        return tm.hindexed([spec[1]] * len(spec[2]), spec[2], oracle_type(spec[3]))
    if kind == "struct":
        return tm.struct(spec[1], spec[2], [oracle_type(t) for t in spec[3]])
    if kind == "resized":
        return tm.resized(oracle_type(spec[1]), spec[2], spec[3])
    if kind == "dup":
        return oracle_type(spec[1])
    if kind == "subarray":
        return tm.subarray(spec[1], spec[2], spec[3], spec[4] == 56, oracle_type(spec[5]))
    raise ValueError(kind)


B = lambda h: ("builtin", h)  # noqa: E731

# (name, spec, count)
CASES = [
    ("vector_int_simple_pack", ("vector", 8, 1, 2, B(INT)), 1),
    ("vector_float_cfg5", ("vector", 4096, 4, 8, B(FLOAT)), 1),
    ("vector_count3", ("vector", 5, 3, 7, B(FLOAT)), 3),
    ("vecblklen", ("vector", 17, 9, 11, B(CHAR)), 2),
    ("zero_blklen_vector", ("vector", 6, 0, 3, B(INT)), 2),
    ("slice_vec_of_vec", ("vector", 4, 1, 3, ("vector", 5, 2, 4, B(DOUBLE))), 2),
    ("hvector_neg_gap", ("hvector", 4, 2, 24, B(SHORT)), 5),
    ("contig_of_vector", ("contiguous", 3, ("vector", 4, 1, 2, B(FLOAT))), 2),
    ("indexed_ragged", ("indexed", [3, 0, 1, 5, 2], [0, 4, 5, 9, 20], B(INT)), 4),
    ("indexed_unsorted", ("indexed", [2, 2, 1], [10, 0, 5], B(DOUBLE)), 3),
    ("hindexed_bytes", ("hindexed", [1, 7, 2], [3, 9, 40], B(CHAR)), 6),
    ("indexed_block", ("indexed_block", 3, [0, 6, 7, 20], B(FLOAT)), 3),
    ("hindexed_block", ("hindexed_block", 2, [0, 24, 56], B(DOUBLE)), 2),
    ("pair_double_int", B(DOUBLE_INT), 33),
    ("pair_short_int", B(SHORT_INT), 21),
    ("pair_long_int", B(LONG_INT), 9),
    ("struct_double_int_padded", ("struct", [1, 1], [0, 8], [B(DOUBLE), B(INT)]), 7),
    ("struct_char_double", ("struct", [1, 2], [0, 8], [B(CHAR), B(DOUBLE)]), 5),
    ("struct_nested", ("struct", [2, 1, 3], [0, 16, 40], [B(SHORT), ("vector", 2, 1, 2, B(INT)), B(CHAR)]), 4),
    ("struct_zero_len_block", ("struct", [1, 0, 2], [0, 100, 4], [B(INT), B(DOUBLE), B(SHORT)]), 3),
    ("resized_vector", ("resized", ("vector", 3, 1, 2, B(INT)), 0, 48), 4),
    ("resized_lb_shift", ("resized", ("contiguous", 2, B(SHORT)), -4, 12), 5),
    ("dup_of_indexed", ("dup", ("indexed", [1, 2], [1, 4], B(FLOAT))), 3),
    ("subarray_2d_c", ("subarray", [8, 10], [3, 4], [2, 5], 56, B(FLOAT)), 2),
    ("subarray_3d_c", ("subarray", [5, 6, 7], [2, 3, 4], [1, 2, 3], 56, B(DOUBLE)), 1),
    ("subarray_2d_fortran", ("subarray", [8, 10], [3, 4], [2, 5], 57, B(INT)), 2),
    ("subarray_of_pairs", ("subarray", [4, 6], [2, 3], [1, 1], 56, B(DOUBLE_INT)), 1),
]
