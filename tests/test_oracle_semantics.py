"""Targeted semantics of the oracle (reference file:line in each assertion)."""
import numpy as np
import pytest

from mvapich2_amd.consts import OPS, TYPES, legal_pairs, DEVICE_UNSUPPORTED
from oracle import oracle


def rl(tname, op, a, b):
    """inout=a, in=b -> op(a, b)"""
    a = np.array(a, dtype=TYPES[tname][1] if isinstance(TYPES[tname][1], str) else TYPES[tname][1])
    b = np.array(b, dtype=a.dtype)
    assert oracle.reduce_local(b, a, len(a), TYPES[tname][0], OPS[op]) == 0
    return a


def bits(x):
    return np.array(x).view(np.uint32 if np.array(x).dtype == np.float32 else np.uint64)


def test_max_min_nan_and_signed_zero():
    # MPIR_MAX/MPIR_MIN mpiimpl.h:4034-4040: NaN is skipped, ties keep a (inoutvec)
    nan = np.float32(np.nan)
    r = rl("MPI_FLOAT", "MPI_MAX", [nan, 1.0, nan, -0.0, 0.0], [2.0, nan, nan, 0.0, -0.0])
    assert r[0] == 2.0 and r[1] == 1.0 and np.isnan(r[2])
    assert np.signbit(r[3]) and not np.signbit(r[4])  # tie keeps a
    r = rl("MPI_DOUBLE", "MPI_MIN", [np.nan, -0.0, 3.0], [5.0, 0.0, 2.0])
    assert r[0] == 5.0 and np.signbit(r[1]) and r[2] == 2.0


def test_logical_ops_store_zero_one_in_float():
    # opland.c:73-76 floats allowed, result 0/1 in the element type
    r = rl("MPI_FLOAT", "MPI_LAND", [2.5, 0.0, np.nan], [3.0, 1.0, 1.0])
    assert list(r) == [1.0, 0.0, 1.0]
    r = rl("MPI_DOUBLE", "MPI_LXOR", [2.5, 0.0, 0.0], [3.0, 1.0, 0.0])
    assert list(r) == [0.0, 1.0, 0.0]


def test_integer_sum_prod_wrap():
    r = rl("MPI_INT", "MPI_SUM", [2**31 - 1], [1])
    assert r[0] == -(2**31)
    r = rl("MPI_UNSIGNED_SHORT", "MPI_PROD", [65535], [65535])
    assert r[0] == 1
    r = rl("MPI_SIGNED_CHAR", "MPI_PROD", [100], [3])
    assert r[0] == np.int8(300 - 256)


def test_maxloc_minloc_ties_and_nan():
    # opmaxloc.c:65-87: a<b -> b; equal -> loc = min; NaN handling
    dt = np.dtype([("value", "f4"), ("loc", "i4")])
    a = np.array([(1.0, 5), (2.0, 3), (np.nan, 7), (1.0, 2), (np.nan, 9)], dtype=dt)
    b = np.array([(1.0, 2), (1.0, 0), (3.0, 1), (np.nan, 0), (np.nan, 4)], dtype=dt)
    assert oracle.reduce_local(b, a, 5, TYPES["MPI_FLOAT_INT"][0], OPS["MPI_MAXLOC"]) == 0
    assert list(a["loc"]) == [2, 3, 1, 2, 4]
    assert a["value"][2] == 3.0 and np.isnan(a["value"][4])


def test_complex_c99_annex_g_recovery():
    # C99 _Complex multiply (gcc -> __mulsc3): (inf + nan i) * (1 + 0i) recovers an infinity
    a = np.array([complex(np.inf, np.nan)], dtype=np.complex64)
    b = np.array([complex(1.0, 0.0)], dtype=np.complex64)
    assert oracle.reduce_local(b, a, 1, TYPES["MPI_C_FLOAT_COMPLEX"][0], OPS["MPI_PROD"]) == 0
    assert np.isinf(a[0].real)
    # Fortran COMPLEX uses the plain struct formula (opprod.c:50-51): no recovery
    a = np.array([complex(np.inf, np.nan)], dtype=np.complex64)
    assert oracle.reduce_local(b, a, 1, TYPES["MPI_COMPLEX"][0], OPS["MPI_PROD"]) == 0
    assert np.isnan(a[0].real)


def test_op_check_table():
    legal = set(legal_pairs())
    for op in OPS:
        for t, (h, *_r) in TYPES.items():
            rc = oracle.op_check(OPS[op], h)
            if op in ("MPI_REPLACE", "MPI_NO_OP"):
                assert rc == 0
            elif t == "MPI_WCHAR":
                assert rc == 9
            else:
                assert (rc == 0) == ((op, t) in legal), (op, t)


def test_rs_owner_is_bit_reversed_block():
    """In pt2pt_rs (allreduce_osu.c:853-947) block b is reduced by newrank bitrev(b):
    with MAX on +/-0 the surviving sign tells which rank's operand was the left one."""
    n, count = 8, 8
    for b in range(8):
        sends = []
        for r in range(n):
            x = np.zeros(count, dtype=np.float32)
            x[b] = -0.0 if r == int(f"{b:03b}"[::-1], 2) else 0.0
            sends.append(x)
        outs = oracle.allreduce(sends, count, TYPES["MPI_FLOAT"][0], OPS["MPI_MAX"], 2)
        for r in range(n):
            assert np.signbit(outs[r][b]), (b, r)


def test_pack_roundtrip():
    src = np.arange(64, dtype=np.uint8)
    p = oracle.pack_strided(src, 4, 4, 16)
    assert list(p[:8]) == [0, 1, 2, 3, 16, 17, 18, 19]
    dst = np.zeros(64, dtype=np.uint8)
    oracle.unpack_strided(p, dst, 4, 4, 16)
    assert np.array_equal(dst.reshape(4, 16)[:, :4], src.reshape(4, 16)[:, :4])
    assert not dst.reshape(4, 16)[:, 4:].any()


def test_reduce_scatter_ring_order():
    """MPIR_Reduce_scatter_ring (red_scat_osu.c:1026-1180): block b = op(x_b, op(x_{b-1}, ...
    op(x_{b+2}, x_{b+1}))) with each hop's own operand as the accumulator."""
    import numpy as np
    from mvapich2_amd.consts import OPS, TYPES
    from oracle import oracle
    n, c = 3, 2
    # fp32 values whose sum depends on association order
    xs = [np.array([1e8, 1.0, 1.0, -1e8, 3.0, 7.0], dtype=np.float32),
          np.array([1.0, 1e8, -1e8, 1.0, 5.0, 11.0], dtype=np.float32),
          np.array([-1e8, -1e8, 1e8, 1e8, 13.0, 17.0], dtype=np.float32)]
    got = oracle.reduce_scatter_ring(xs, [c] * n, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"])
    want = np.zeros(n * c, dtype=np.float32)
    for b in range(n):
        blk = slice(b * c, (b + 1) * c)
        acc = xs[(b + 1) % n][blk].copy()
        for k in range(2, n + 1):
            acc = (xs[(b + k) % n][blk] + acc).astype(np.float32)
        want[blk] = acc
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    # integers: any order gives the linear result
    xi = [np.arange(12, dtype=np.int32) * (r + 1) for r in range(4)]
    ring = oracle.reduce_scatter_ring(xi, [3] * 4, TYPES["MPI_INT"][0], OPS["MPI_SUM"])
    lin = oracle.reduce_linear(xi, 12, TYPES["MPI_INT"][0], OPS["MPI_SUM"])
    assert np.array_equal(ring, lin)
