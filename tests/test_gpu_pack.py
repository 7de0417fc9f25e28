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
