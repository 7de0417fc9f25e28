"""Part (3) parity: device pack / unpack of strided layouts (MPI_Type_vector
family) vs the oracle's segment copy (segment_packunpack.c:175-305)."""
import ctypes

import numpy as np
import pytest

import mvapich2_amd as m
from mvapich2_amd.consts import TYPES
from oracle import oracle

pytestmark = pytest.mark.gpu

SHAPES = [(1, 4, 4), (1000, 4, 8), (1000, 4, 32), (777, 16, 48), (100, 12, 40), (4096, 1, 3), (333, 64, 64),
          (10000, 2, 6), (50, 1000, 1024), (3, 7, 9)]


@pytest.mark.parametrize("nb,blk,stride", SHAPES)
def test_pack_unpack_strided(nb, blk, stride):
    L = m.lib()
    rng = np.random.default_rng(nb * 7 + blk)
    span = (nb - 1) * stride + blk
    src = rng.integers(0, 256, span + 64, dtype=np.uint8)
    for off in (0, 4, 3):
        d_src = m.DeviceBuffer.from_array(src)
        d_pk = m.DeviceBuffer(nb * blk + 64)
        assert L.mv2h_pack_strided(d_src.ptr + off, d_pk.ptr, nb, blk, stride, None) == 0
        got = d_pk.download(np.uint8, count=nb * blk)
        want = oracle.pack_strided(src[off:].copy(), nb, blk, stride)
        assert np.array_equal(got, want), (nb, blk, stride, off)
        # unpack into a canvas: gap bytes must be untouched
        canvas = rng.integers(0, 256, span + 64, dtype=np.uint8)
        d_can = m.DeviceBuffer.from_array(canvas)
        assert L.mv2h_unpack_strided(d_pk.ptr, d_can.ptr + off, nb, blk, stride, None) == 0
        got = d_can.download(np.uint8)
        w2 = canvas.copy()
        tmp = w2[off:].copy()
        oracle.unpack_strided(oracle.pack_strided(src[off:].copy(), nb, blk, stride), tmp, nb, blk, stride)
        w2[off:] = tmp
        assert np.array_equal(got, w2), ("unpack", nb, blk, stride, off)


def test_mpi_pack_vector_type_device_and_host():
    """MPI_Type_vector(N, 4, 8, MPI_FLOAT) (BASELINE config 5 operand) through
    MPI_Pack / MPI_Unpack on device buffers, and the host-buffer path."""
    L = m.lib()
    N = 10000
    vt = ctypes.c_int()
    assert L.MPI_Type_vector(N, 4, 8, TYPES["MPI_FLOAT"][0], ctypes.byref(vt)) == 0
    assert L.MPI_Type_commit(ctypes.byref(vt)) == 0
    size = ctypes.c_int()
    assert L.MPI_Type_size(vt.value, ctypes.byref(size)) == 0 and size.value == N * 16
    lb, ext = ctypes.c_long(), ctypes.c_long()
    assert L.MPI_Type_get_extent(vt.value, ctypes.byref(lb), ctypes.byref(ext)) == 0
    assert ext.value == ((N - 1) * 8 + 4) * 4
    x = np.arange(N * 8, dtype=np.float32)
    want = x.reshape(N, 8)[:, :4].ravel()
    for device in (True, False):
        if device:
            src = m.DeviceBuffer.from_array(x)
            out = m.DeviceBuffer(N * 16)
            sp, op = src.ptr, out.ptr
        else:
            hout = np.zeros(N * 4, dtype=np.float32)
            sp, op = x.ctypes.data, hout.ctypes.data
        pos = ctypes.c_int(0)
        assert L.MPI_Pack(sp, 1, vt.value, op, N * 16, ctypes.byref(pos), 0x44000000) == 0
        assert pos.value == N * 16
        got = out.download(np.float32) if device else hout
        assert np.array_equal(got, want)
    # unpack back into a -1 canvas: gaps untouched
    canvas = m.DeviceBuffer.from_array(np.full(N * 8, -1.0, dtype=np.float32))
    pk = m.DeviceBuffer.from_array(want)
    pos = ctypes.c_int(0)
    assert L.MPI_Unpack(pk.ptr, N * 16, ctypes.byref(pos), canvas.ptr, 1, vt.value, 0x44000000) == 0
    got = canvas.download(np.float32).reshape(N, 8)
    assert np.array_equal(got[:, :4].ravel(), want) and np.all(got[:, 4:] == -1.0)
    assert L.MPI_Type_free(ctypes.byref(vt)) == 0


# ---- any flattened layout: the run-table kernel (mv2h_pack_segments) ----
from oracle import typemap as tm  # noqa: E402
from tests.typecases import CASES, Built, oracle_type  # noqa: E402


def _segments(rng, nseg, align):
    offs, lens, pos = [], [], int(rng.integers(0, 3)) * align
    for _ in range(nseg):
        pos += int(rng.integers(0, 4)) * align
        ln = int(rng.integers(1, 6)) * align
        offs.append(pos)
        lens.append(ln)
        pos += ln
    return offs, lens, pos


@pytest.mark.parametrize("seed", range(12))
def test_pack_segments_random_tables(seed):
    """Random run tables (unit sizes 1..16 B, 1..700 segments so that the LDS
    table and the global-memory table are both used) vs the oracle walk."""
    L = m.lib()
    rng = np.random.default_rng(100 + seed)
    align = [1, 2, 4, 8, 16, 16][seed % 6]
    nseg = [1, 3, 40, 700][seed % 4]
    offs, lens, end = _segments(rng, nseg, align)
    extent = end + int(rng.integers(0, 3)) * align
    count = int(rng.integers(1, 300))
    span = (count - 1) * extent + end
    src = rng.integers(0, 256, span + 32, dtype=np.uint8)
    packed_n = count * sum(lens)
    want = np.zeros(packed_n, dtype=np.uint8)
    oracle.pack_segments(src, want, count, extent, offs, lens)
    o64 = (ctypes.c_int64 * nseg)(*offs)
    l64 = (ctypes.c_int64 * nseg)(*lens)
    d_src = m.DeviceBuffer.from_array(src)
    d_pk = m.DeviceBuffer(packed_n + 16)
    assert L.mv2h_pack_segments(d_src.ptr, d_pk.ptr, count, extent, o64, l64, nseg, 0, None) == 0
    assert np.array_equal(d_pk.download(np.uint8, count=packed_n), want), (seed, align, nseg)
    canvas = rng.integers(0, 256, span + 32, dtype=np.uint8)
    d_can = m.DeviceBuffer.from_array(canvas)
    assert L.mv2h_pack_segments(d_pk.ptr, d_can.ptr, count, extent, o64, l64, nseg, 1, None) == 0
    w2 = canvas.copy()
    oracle.pack_segments(want, w2, count, extent, offs, lens, unpack=True)
    assert np.array_equal(d_can.download(np.uint8), w2), ("unpack", seed)


@pytest.mark.parametrize("name,spec,count", CASES, ids=[c[0] for c in CASES])
def test_device_mpi_pack_unpack_all_type_shapes(name, spec, count):
    """MPI_Pack / MPI_Unpack on device buffers for every derived-type shape of
    the reference's datatype tests, vs the type-map oracle; also the mixed
    host/device directions."""
    L = m.lib()
    b = Built(L)
    try:
        h = b.lib_type(spec)
        assert L.MPI_Type_commit(ctypes.byref(ctypes.c_int(h))) == 0
        t = oracle_type(spec)
        if not t.size:
            return
        span = (count - 1) * t.extent + t.true_lb + t.true_extent
        rng = np.random.default_rng(len(name) * 31)
        src = rng.integers(0, 256, span + 16, dtype=np.uint8)
        psize = count * t.size
        want = tm.pack(src, t, count)
        d_src = m.DeviceBuffer.from_array(src)
        d_out = m.DeviceBuffer(psize + 8)
        pos = ctypes.c_int(0)
        assert L.MPI_Pack(d_src.ptr, count, h, d_out.ptr, psize + 8, ctypes.byref(pos), 0x44000000) == 0
        assert pos.value == psize
        assert np.array_equal(d_out.download(np.uint8, count=psize), want), name
        # device source -> host packed
        hout = np.zeros(psize, dtype=np.uint8)
        pos = ctypes.c_int(0)
        assert L.MPI_Pack(d_src.ptr, count, h, hout.ctypes.data, psize, ctypes.byref(pos), 0x44000000) == 0
        assert np.array_equal(hout, want), ("d->h", name)
        canvas = rng.integers(0, 256, span + 16, dtype=np.uint8)
        d_can = m.DeviceBuffer.from_array(canvas)
        pos = ctypes.c_int(0)
        assert L.MPI_Unpack(d_out.ptr, psize, ctypes.byref(pos), d_can.ptr, count, h, 0x44000000) == 0
        assert np.array_equal(d_can.download(np.uint8), tm.unpack(want, canvas, t, count)), ("unpack", name)
        # host packed -> device destination
        d_can2 = m.DeviceBuffer.from_array(canvas)
        pos = ctypes.c_int(0)
        assert L.MPI_Unpack(want.ctypes.data, psize, ctypes.byref(pos), d_can2.ptr, count, h, 0x44000000) == 0
        assert np.array_equal(d_can2.download(np.uint8), tm.unpack(want, canvas, t, count)), ("h->d", name)
    finally:
        b.close()
