"""x87 80-bit long double types (MPI_LONG_DOUBLE, MPI_C_LONG_DOUBLE_COMPLEX,
MPI_LONG_DOUBLE_INT): gfx950 has no 80-bit float, so the library reduces them
on the host with its own loops (mpi_api.cpp ld_uop), like the reference's
(oputil.h:316-349, opmaxloc.c:65-87).  Host-buffer MPI_Reduce_local here is
host logic only (no GPU call); the -m gpu tests run the same types through the
collectives with device buffers."""
import numpy as np
import pytest

import mvapich2_amd as m
from mvapich2_amd.consts import OPS
from oracle import oracle

# name -> (handle, extent); include/mpi.h
X87_TYPES = {"MPI_LONG_DOUBLE": (0x4C00100C, 16), "MPI_C_LONG_DOUBLE_COMPLEX": (0x4C002042, 32),
             "MPI_LONG_DOUBLE_INT": (0x8C000004, 32)}
X87 = list(X87_TYPES)


def x87_operand(t, count, rng):
    if t == "MPI_LONG_DOUBLE":
        x = (rng.standard_normal(count) * 10.0 ** rng.uniform(-3, 3, count)).astype(np.longdouble)
        x[:6] = [np.nan, -0.0, 0.0, np.inf, -np.inf, 1.0]
        return x.view(np.uint8).ravel().copy()
    if t == "MPI_C_LONG_DOUBLE_COMPLEX":
        x = (rng.standard_normal(count) + 1j * rng.standard_normal(count)).astype(np.clongdouble)
        x[:3] = [complex(np.inf, np.nan), complex(np.nan, np.inf), complex(0.0, -0.0)]
        return x.view(np.uint8).ravel().copy()
    dt = np.dtype([("value", np.longdouble), ("loc", "<i4"), ("pad", "<i4", 3)])
    x = np.zeros(count, dt)
    x["value"] = np.floor(rng.uniform(-4, 4, count))
    x["value"][:2] = np.nan
    x["loc"] = rng.integers(0, 8, count)
    return x.view(np.uint8).ravel().copy()


@pytest.mark.parametrize("t", X87)
def test_x87_reduce_local_host_matches_oracle(t):
    L = m.lib()
    h, ext = X87_TYPES[t]
    rng = np.random.default_rng(87)
    count = 1001
    ops = [op for op in OPS if op not in ("MPI_REPLACE", "MPI_NO_OP") and oracle.op_check(OPS[op], h) == 0]
    assert ops
    for op in ops:
        a, b = x87_operand(t, count, rng), x87_operand(t, count, rng)
        want = b.copy()
        assert oracle.reduce_local(a, want, count, h, OPS[op]) == 0
        got = b.copy()
        assert L.MPI_Reduce_local(a.ctypes.data, got.ctypes.data, count, h, OPS[op]) == 0
        if t == "MPI_LONG_DOUBLE_INT":  # value (10 bytes of x87) + loc; padding is not data
            g, w = got.reshape(count, 32), want.reshape(count, 32)
            assert np.array_equal(g[:, :10], w[:, :10]) and np.array_equal(g[:, 16:20], w[:, 16:20]), op
        else:
            gv, wv = got.reshape(-1, 16)[:, :10], want.reshape(-1, 16)[:, :10]  # x87 value bytes
            assert np.array_equal(gv, wv), (t, op)
