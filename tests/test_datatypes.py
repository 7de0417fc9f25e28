"""Derived datatypes on the host path (no GPU): every constructor's size /
lb / extent / true extent and the MPI_Pack / MPI_Unpack byte streams equal
the type-map oracle (oracle/typemap.py), for the reference's datatype test
shapes (tests/typecases.py).  The device path runs the same cases in
tests/test_gpu_pack.py."""
import ctypes

import numpy as np
import pytest

import mvapich2_amd as m
from oracle import oracle
from oracle import typemap as tm
from tests.typecases import CASES, Built, oracle_type

COMM_WORLD = 0x44000000


@pytest.mark.parametrize("name,spec,count", CASES, ids=[c[0] for c in CASES])
def test_type_bounds_match_oracle(name, spec, count):
    L = m.lib()
    b = Built(L)
    try:
        h = b.lib_type(spec)
        want = oracle_type(spec)
        size = ctypes.c_int()
        lb, ext, tlb, text = (ctypes.c_long() for _ in range(4))
        assert L.MPI_Type_size(h, ctypes.byref(size)) == 0
        assert L.MPI_Type_get_extent(h, ctypes.byref(lb), ctypes.byref(ext)) == 0
        assert L.MPI_Type_get_true_extent(h, ctypes.byref(tlb), ctypes.byref(text)) == 0
        assert (size.value, lb.value, ext.value) == (want.size, want.lb, want.extent), name
        if want.size:
            assert (tlb.value, text.value) == (want.true_lb, want.true_extent), name
    finally:
        b.close()


@pytest.mark.parametrize("name,spec,count", CASES, ids=[c[0] for c in CASES])
def test_host_pack_unpack_match_oracle(name, spec, count):
    L = m.lib()
    b = Built(L)
    try:
        h = b.lib_type(spec)
        assert L.MPI_Type_commit(ctypes.byref(ctypes.c_int(h))) == 0
        t = oracle_type(spec)
        span = (count - 1) * t.extent + t.true_lb + t.true_extent if t.size else 0
        rng = np.random.default_rng(len(name))
        src = rng.integers(0, 256, span + 16, dtype=np.uint8)
        psize = count * t.size
        out = np.zeros(psize + 8, dtype=np.uint8)
        pos = ctypes.c_int(0)
        assert L.MPI_Pack(src.ctypes.data, count, h, out.ctypes.data, psize + 8, ctypes.byref(pos), COMM_WORLD) == 0
        assert pos.value == psize
        assert np.array_equal(out[:psize], tm.pack(src, t, count)), name
        canvas = rng.integers(0, 256, span + 16, dtype=np.uint8)
        got = canvas.copy()
        pos = ctypes.c_int(0)
        assert L.MPI_Unpack(out.ctypes.data, psize, ctypes.byref(pos), got.ctypes.data, count, h, COMM_WORLD) == 0
        assert np.array_equal(got, tm.unpack(out[:psize], canvas, t, count)), name
    finally:
        b.close()


@pytest.mark.parametrize("name,spec,count", CASES, ids=[c[0] for c in CASES])
def test_segment_oracle_agrees_with_typemap_oracle(name, spec, count):
    """The C segment-walk oracle (used for the device kernel) and the Python
    type-map oracle describe the same byte stream."""
    t = oracle_type(spec)
    if not t.entries:
        return
    span = (count - 1) * t.extent + t.true_lb + t.true_extent
    src = np.random.default_rng(3).integers(0, 256, span + 16, dtype=np.uint8)
    offs = [d for d, _ in t.entries]
    lens = [n for _, n in t.entries]
    dst = np.zeros(count * t.size, dtype=np.uint8)
    oracle.pack_segments(src, dst, count, t.extent, offs, lens)
    assert np.array_equal(dst, tm.pack(src, t, count))
    canvas = np.random.default_rng(4).integers(0, 256, span + 16, dtype=np.uint8)
    back = canvas.copy()
    oracle.pack_segments(dst, back, count, t.extent, offs, lens, unpack=True)
    assert np.array_equal(back, tm.unpack(dst, canvas, t, count))


def test_struct_padding_rules():
    """pairtype-size-extent.c: {double, int} struct pads to 16 like MPI_DOUBLE_INT;
    {char, double} pads to 16; {short, char} to 4."""
    for spec, ext in ((("struct", [1, 1], [0, 8], [("builtin", 0x4c00080b), ("builtin", 0x4c000405)]), 16),
                      (("struct", [1, 1], [0, 2], [("builtin", 0x4c000203), ("builtin", 0x4c000101)]), 4)):
        L = m.lib()
        b = Built(L)
        h = b.lib_type(spec)
        lb, e = ctypes.c_long(), ctypes.c_long()
        assert L.MPI_Type_get_extent(h, ctypes.byref(lb), ctypes.byref(e)) == 0
        assert e.value == ext == oracle_type(spec).extent
        b.close()


def test_negative_data_displacement_is_rejected():
    L = m.lib()
    h = ctypes.c_int()
    assert L.MPI_Type_create_hvector(3, 1, -8, 0x4c000405, ctypes.byref(h)) == 12  # MPI_ERR_ARG
