"""Part (1) parity: MPI_Reduce_local / mv2h_reduce_local on device buffers vs
the oracle, bit-exact for every (op, type) pair the reference accepts."""
import numpy as np
import pytest

import mvapich2_amd as m
from mvapich2_amd.consts import DEVICE_UNSUPPORTED, OPS, TYPES, legal_pairs
from oracle import oracle
from tests.helpers import as_bytes, assert_bytes_equal, rand_typed

pytestmark = pytest.mark.gpu
PAIRS = [(op, t) for op, t in legal_pairs() if t not in DEVICE_UNSUPPORTED]


def run_rl(tname, op, x, y, count, off=0):
    """device: y <- op(y, x) with both operands shifted by `off` elements."""
    ext = TYPES[tname][3]
    a = m.DeviceBuffer((count + off) * ext)
    b = m.DeviceBuffer((count + off) * ext)
    a.upload(x, off * ext)
    b.upload(y, off * ext)
    rc = m.lib().MPI_Reduce_local(a.ptr + off * ext, b.ptr + off * ext, count, TYPES[tname][0], OPS[op])
    assert rc == 0, (tname, op, rc)
    return b.download(np.uint8, count=count * ext, offset=off * ext)


@pytest.mark.parametrize("count", [1, 7, 1000, 4099])
def test_all_pairs_bit_exact(count):
    rng = np.random.default_rng(count)
    for op, t in PAIRS:
        small = op == "MPI_PROD"
        x = rand_typed(t, count, rng, small=small)
        y = rand_typed(t, count, rng, small=small)
        want = y.copy()
        assert oracle.reduce_local(x, want, count, TYPES[t][0], OPS[op]) == 0
        for off in (0, 1):
            got = run_rl(t, op, x, y, count, off)
            assert_bytes_equal(got, want, t, count, f"{op} off={off}")


def test_reduce_local_c_known_answers(golden):
    cases, arrs = golden
    for c in cases:
        if c["family"] != "reduce_local":
            continue
        ins = arrs[c["id"] + "__in"]
        sol = arrs[c["id"] + "__sol"]
        if c["count"] == 0:
            continue
        got = run_rl("MPI_INT", "MPI_SUM", ins[0].view(np.int32), ins[1].view(np.int32), c["count"])
        assert np.array_equal(got, sol), c["id"]


def test_count_zero_and_replace_no_op():
    L = m.lib()
    a = m.DeviceBuffer.from_array(np.arange(16, dtype=np.int32))
    b = m.DeviceBuffer.from_array(np.full(16, 7, dtype=np.int32))
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 0, TYPES["MPI_INT"][0], OPS["MPI_SUM"]) == 0
    assert np.all(b.download(np.int32) == 7)
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 16, TYPES["MPI_INT"][0], OPS["MPI_NO_OP"]) == 0
    assert np.all(b.download(np.int32) == 7)
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 16, TYPES["MPI_INT"][0], OPS["MPI_REPLACE"]) == 0
    assert np.array_equal(b.download(np.int32), np.arange(16))


def test_errors_are_mpi_classes():
    L = m.lib()
    L.MPI_Comm_set_errhandler(0x44000000, 0x54000001)  # MPI_ERRORS_RETURN
    a = m.DeviceBuffer(64)
    b = m.DeviceBuffer(64)
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 4, TYPES["MPI_FLOAT"][0], OPS["MPI_BAND"]) == 9  # MPI_ERR_OP
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 4, TYPES["MPI_INT"][0], OPS["MPI_MAXLOC"]) == 9
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 4, 0x1234, OPS["MPI_SUM"]) == 3    # MPI_ERR_TYPE
    assert L.MPI_Reduce_local(a.ptr, b.ptr, -1, TYPES["MPI_INT"][0], OPS["MPI_SUM"]) == 2
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 1, TYPES["MPI_LONG_DOUBLE"][0], OPS["MPI_BAND"]) == 9


def test_x87_long_double_device_buffers():
    """MPI_LONG_DOUBLE has no gfx950 representation: device operands are staged through the
    host and reduced there in 80-bit x87 (mpi_api.cpp ld_uop), not rejected."""
    L = m.lib()
    x = (np.arange(100, dtype=np.longdouble) / 3).astype(np.longdouble)
    y = np.full(100, np.longdouble(1) / 7, dtype=np.longdouble)
    a, b = m.DeviceBuffer.from_array(x), m.DeviceBuffer.from_array(y)
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 100, TYPES["MPI_LONG_DOUBLE"][0], OPS["MPI_SUM"]) == 0
    assert np.array_equal(b.download(np.longdouble), x + y)


def test_host_buffers_are_reduced_on_the_gpu():
    x = np.arange(1000, dtype=np.float64)
    y = np.ones(1000, dtype=np.float64)
    assert m.lib().MPI_Reduce_local(x.ctypes.data, y.ctypes.data, 1000, TYPES["MPI_DOUBLE"][0], OPS["MPI_SUM"]) == 0
    assert np.array_equal(y, np.arange(1000) + 1.0)


def test_user_op_non_commutative():
    """reduce_local.c user_op: inout = 2*in + inout (non-commutative), device buffers."""
    import ctypes
    L = m.lib()
    FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))

    def uop(inp, io, ln, dt):
        n = ln[0]
        a = np.ctypeslib.as_array((ctypes.c_int * n).from_address(inp))
        b = np.ctypeslib.as_array((ctypes.c_int * n).from_address(io))
        b[:] = a * 2 + b
    cb = FN(uop)
    op = ctypes.c_int()
    assert L.MPI_Op_create(ctypes.cast(cb, ctypes.c_void_p), 0, ctypes.byref(op)) == 0
    count = 1
    while count < 65000:
        i = np.arange(count, dtype=np.int32)
        a, b = m.DeviceBuffer.from_array(i), m.DeviceBuffer.from_array(i)
        assert L.MPI_Reduce_local(a.ptr, b.ptr, count, TYPES["MPI_INT"][0], op.value) == 0
        assert np.array_equal(b.download(np.int32), 3 * i)
        count *= 2
    assert L.MPI_Op_free(ctypes.byref(op)) == 0


@pytest.mark.parametrize("tname,op", [("MPI_FLOAT", "MPI_SUM"), ("MPI_FLOAT", "MPI_MAX"), ("MPI_INT", "MPI_SUM"),
                                      ("MPI_DOUBLE", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MAX")])
def test_full_size_256MiB(tname, op):
    """BASELINE config 2 sizes: each output element is one IEEE op / one integer
    op, so numpy's elementwise result is the exact expected value."""
    dt = m.np_dtype(tname)
    count = 256 * 1024 * 1024 // dt.itemsize
    rng = np.random.default_rng(0x5EED)
    if dt.kind == "f":
        x = rng.uniform(-1, 1, count).astype(dt)
        y = rng.uniform(-1, 1, count).astype(dt)
    else:
        x = rng.integers(-(2**31), 2**31 - 1, count, dtype=np.int64).astype(dt)
        y = rng.integers(-(2**31), 2**31 - 1, count, dtype=np.int64).astype(dt)
    a, b = m.DeviceBuffer.from_array(x), m.DeviceBuffer.from_array(y)
    assert m.lib().MPI_Reduce_local(a.ptr, b.ptr, count, TYPES[tname][0], OPS[op]) == 0
    got = b.download(dt)
    with np.errstate(over="ignore"):
        want = (x + y) if op == "MPI_SUM" else np.maximum(x, y)
    assert np.array_equal(got, want)


def test_op_table_entries_on_device_buffers():
    """include/mpir_op.h: MPIR_OP_HDL_TO_FN(op)(in, inout, &len, &type) on device buffers gives
    MPI_Reduce_local's bits (MPIR_Op_table, allreduce.c:95-100); a type the op rejects leaves
    inoutvec untouched and MPIR_Op_errno() returns MPI_ERR_OP (opsum.c:82-86)."""
    import ctypes
    L = m.lib()
    table = (ctypes.c_void_p * 14).in_dll(L, "MPIR_Op_table")
    UF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                          ctypes.POINTER(ctypes.c_int))
    rng = np.random.default_rng(4031)
    count = 3001
    for op, t in PAIRS:
        x = rand_typed(t, count, rng, small=op == "MPI_PROD")
        y = rand_typed(t, count, rng, small=op == "MPI_PROD")
        want = y.copy()
        assert oracle.reduce_local(x, want, count, TYPES[t][0], OPS[op]) == 0
        a, b = m.DeviceBuffer.from_array(x), m.DeviceBuffer.from_array(y)
        n, ty = ctypes.c_int(count), ctypes.c_int(TYPES[t][0])
        UF(table[(OPS[op] & 0xF) - 1])(a.ptr, b.ptr, ctypes.byref(n), ctypes.byref(ty))
        assert L.MPIR_Op_errno() == 0, (op, t)
        assert_bytes_equal(b.download(np.uint8), as_bytes(want), t, count, f"MPIR_Op_table {op}")
    a, b = m.DeviceBuffer.from_array(np.ones(16, np.float32)), m.DeviceBuffer.from_array(np.full(16, 5, np.float32))
    n, ty = ctypes.c_int(16), ctypes.c_int(TYPES["MPI_FLOAT"][0])
    UF(table[(OPS["MPI_BXOR"] & 0xF) - 1])(a.ptr, b.ptr, ctypes.byref(n), ctypes.byref(ty))
    assert L.MPIR_Op_errno() == 9
    assert L.MPIR_Op_errno() == 0
    assert np.all(b.download(np.float32) == 5)


def test_result_visible_to_a_copy_engine_at_return():
    """A blocking call returns on the kernel-written completion word, before the kernel's own
    end-of-kernel release; the result must nevertheless be in memory for any reader at that point
    (device_util.h block_done: every XCD's L2 written back before its group counts, r04y).  A copy
    on a non-blocking stream issued right at return — not ordered behind the kernel — reads it;
    SUM of integers with a fresh pattern per round, so a stale line shows as the previous round's
    value.  A guard of the contract, not a reproducer: one run against the pre-fix word passed
    (the race is rare; r04x's failure came from a 12-rank schedule under load)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    st = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0  # hipStreamNonBlocking
    L = m.lib()
    count = 16 << 20  # 64 MiB of int32: every XCD's L2 holds dirty lines of the result
    I32, SUM = TYPES["MPI_INT"][0], OPS["MPI_SUM"]
    a, b, c = m.DeviceBuffer(count * 4), m.DeviceBuffer(count * 4), m.DeviceBuffer(count * 4)
    a.upload(np.ones(count, dtype=np.int32))
    for rnd in range(12):
        b.upload(np.full(count, rnd * 1000, dtype=np.int32))
        L.mv2h_device_synchronize()
        assert L.MPI_Reduce_local(a.ptr, b.ptr, count, I32, SUM) == 0
        assert hip.hipMemcpyAsync(ctypes.c_void_p(c.ptr), ctypes.c_void_p(b.ptr), ctypes.c_size_t(count * 4), 3, st) == 0
        assert hip.hipStreamSynchronize(st) == 0
        got = c.download(np.int32, count=count)
        bad = np.flatnonzero(got != rnd * 1000 + 1)
        assert bad.size == 0, (rnd, bad.size, bad[:4], got[bad[:4]])
    hip.hipStreamDestroy(st)


def test_completion_word_fallbacks_are_counted():
    """A missed completion word is visible: a Reduce_local launched with its word
    withheld completes through the stream fallback with the right bytes and counts done_queried and
    done_missed; a word marked as raised by a kernel whose block groups ran on several XCDs
    completes by stream synchronisation and counts done_xcd_split (runtime/coll.cpp wait_done,
    settle_split; device_util.h block_done)."""
    L = m.lib()
    n = (1 << 20) + 5
    rng = np.random.default_rng(11)
    x = rng.standard_normal(n).astype(np.float32)
    y = rng.standard_normal(n).astype(np.float32)
    want = y.copy()
    assert oracle.reduce_local(x, want, n, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"]) == 0
    before = {k: m.info(k) for k in ("done_queried", "done_late", "done_missed", "done_xcd_split")}
    m.check(L.mv2h_set_tuning(b"withhold_done", 1), "withhold_done")
    got = run_rl("MPI_FLOAT", "MPI_SUM", x, y, n)
    assert np.array_equal(got, want.view(np.uint8))
    assert m.info("done_missed") == before["done_missed"] + 1
    assert m.info("done_queried") >= before["done_queried"] + 1
    m.check(L.mv2h_set_tuning(b"fake_split", 1), "fake_split")
    got = run_rl("MPI_FLOAT", "MPI_SUM", x, y, n)
    assert np.array_equal(got, want.view(np.uint8))
    assert m.info("done_xcd_split") == before["done_xcd_split"] + 1
    # the word path is back: further calls count nothing
    for _ in range(20):
        got = run_rl("MPI_FLOAT", "MPI_SUM", x, y, n)
        assert np.array_equal(got, want.view(np.uint8))
    assert m.info("done_missed") == before["done_missed"] + 1
    assert m.info("done_xcd_split") == before["done_xcd_split"] + 1


def test_small_reduce_local_takes_the_hsa_queue():
    """Small device operands go through the library's own HSA queue (runtime/aql.cpp): the kernel
    objects were found, the calls were dispatched there, and every result is bit-exact with the
    oracle -- interleaved with large calls (HIP launches on the library's stream) on the same
    buffers, so that the two paths' ordering is exercised."""
    L = m.lib()
    assert m.info("nshare") == 1
    rng = np.random.default_rng(5)
    before = m.info("aql_calls")
    p, q = m.DeviceBuffer(8), m.DeviceBuffer(8)
    assert L.MPI_Reduce_local(p.ptr, q.ptr, 2, TYPES["MPI_INT"][0], OPS["MPI_SUM"]) == 0
    assert m.info("aql_acquire") == 1  # a one-rank job: the agent scope
    big = (1 << 20) + 3
    for i, (op, t) in enumerate(PAIRS[::3]):
        count = [1, 2, 7, 64, 100][i % 5]
        small = op == "MPI_PROD"
        x = rand_typed(t, big, rng, small=small)
        y = rand_typed(t, big, rng, small=small)
        ext = TYPES[t][3]
        a, b = m.DeviceBuffer(big * ext), m.DeviceBuffer(big * ext)
        a.upload(x)
        b.upload(y)
        want = y.copy()
        assert oracle.reduce_local(x, want, big, TYPES[t][0], OPS[op]) == 0  # large call: HIP launch
        assert L.MPI_Reduce_local(a.ptr, b.ptr, big, TYPES[t][0], OPS[op]) == 0
        assert oracle.reduce_local(x, want, count, TYPES[t][0], OPS[op]) == 0  # then a small one: the queue
        assert L.MPI_Reduce_local(a.ptr, b.ptr, count, TYPES[t][0], OPS[op]) == 0
        assert_bytes_equal(b.download(np.uint8, count=big * ext), as_bytes(want), t, big, f"{op} {t} count {count}")
    assert m.info("aql_kernels") > 50
    assert m.info("aql_calls") > before


def test_small_reduce_local_orders_after_null_stream_work():
    """The HSA-queue path keeps the HIP path's ordering: operands written by asynchronous work on
    the legacy null stream just before the call (hipMemsetD32Async, stream 0, not waited for), and
    operands rewritten by a host -> device copy after a call of the queue read them (L2 lines of the
    old values must not be served), are both seen by the reduction (runtime/aql.cpp)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    L = m.lib()
    U32, SUM = TYPES["MPI_UNSIGNED"][0], OPS["MPI_SUM"]
    a, b = m.DeviceBuffer(1 << 20), m.DeviceBuffer(64)
    b.upload(np.zeros(16, dtype=np.uint32))
    want = 0
    for i in range(300):
        # a large async memset first, so that the null stream is still busy at the call
        assert hip.hipMemsetD32Async(a.ptr, i + 1, (1 << 20) // 4, None) == 0
        assert L.MPI_Reduce_local(a.ptr, b.ptr, 2, U32, SUM) == 0
        want += i + 1
    assert np.array_equal(b.download(np.uint32, count=2), np.array([want, want], dtype=np.uint32))
    # rewrite the operand by copies between calls of the queue
    before = m.info("aql_calls")
    b.upload(np.zeros(16, dtype=np.uint32))
    want = 0
    for i in range(300):
        a.upload(np.full(4, 1000 + i, dtype=np.uint32))
        assert L.MPI_Reduce_local(a.ptr, b.ptr, 4, U32, SUM) == 0
        want += 1000 + i
        if i % 50 == 0:
            assert np.array_equal(b.download(np.uint32, count=4), np.full(4, want, dtype=np.uint32)), i
    assert np.array_equal(b.download(np.uint32, count=4), np.full(4, want, dtype=np.uint32))
    assert m.info("aql_calls") > before


SYSTEM_ACQUIRE_CHILD = r"""
import ctypes, json, sys
import numpy as np
import mvapich2_amd as m
from mvapich2_amd.consts import OPS, TYPES
from oracle import oracle
from tests.helpers import as_bytes, data_mask, rand_typed
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
L = m.lib()
U32, SUM = TYPES["MPI_UNSIGNED"][0], OPS["MPI_SUM"]
bad = []
a, b = m.DeviceBuffer(1 << 20), m.DeviceBuffer(64)
b.upload(np.zeros(16, dtype=np.uint32))
want = 0
for i in range(300):  # operands written by null-stream work not waited for
    assert hip.hipMemsetD32Async(a.ptr, i + 1, (1 << 20) // 4, None) == 0
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 2, U32, SUM) == 0
    want += i + 1
bad += [] if np.array_equal(b.download(np.uint32, count=2), np.array([want, want], dtype=np.uint32)) else ["memset"]
scope = m.info("aql_acquire")
b.upload(np.zeros(16, dtype=np.uint32))
want = 0
for i in range(300):  # operands rewritten by host -> device copies between calls
    a.upload(np.full(4, 1000 + i, dtype=np.uint32))
    assert L.MPI_Reduce_local(a.ptr, b.ptr, 4, U32, SUM) == 0
    want += 1000 + i
bad += [] if np.array_equal(b.download(np.uint32, count=4), np.full(4, want, dtype=np.uint32)) else ["upload"]
rng = np.random.default_rng(11)
for op, t in (("MPI_SUM", "MPI_FLOAT"), ("MPI_MAX", "MPI_DOUBLE"), ("MPI_BXOR", "MPI_INT"),
              ("MPI_MAXLOC", "MPI_DOUBLE_INT"), ("MPI_PROD", "MPI_C_DOUBLE_COMPLEX")):
    for count in (1, 7, 60):
        ext = TYPES[t][3]
        x, y = rand_typed(t, count, rng, small=op == "MPI_PROD"), rand_typed(t, count, rng, small=op == "MPI_PROD")
        want_b = y.copy()
        assert oracle.reduce_local(x, want_b, count, TYPES[t][0], OPS[op]) == 0
        xa, yb = m.DeviceBuffer(count * ext), m.DeviceBuffer(count * ext)
        xa.upload(x)
        yb.upload(y)
        assert L.MPI_Reduce_local(xa.ptr, yb.ptr, count, TYPES[t][0], OPS[op]) == 0
        mask = data_mask(t, count)  # pair types: the padding bytes carry no value
        if not np.array_equal(yb.download(np.uint8, count=count * ext)[mask], as_bytes(want_b)[mask]):
            bad.append(f"{op} {t} {count}")
print(json.dumps({"scope": scope, "aql_calls": m.info("aql_calls"), "bad": bad}))
"""


def test_small_reduce_local_system_acquire():
    """A job with other ranks dispatches the HSA-queue Reduce_local with the system-scope acquire (a
    peer GPU's stores over xGMI pass none of this GPU's L2s, runtime/aql.cpp).  One GPU cannot hold
    such a job with a rank per GPU, so a fresh process sets that scope with MV2AMD_AQL_ACQUIRE=2 and
    runs the ordering checks of the test above (null-stream writes not waited for, host copies
    between calls) and a bit-exact sweep through it."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MV2AMD_AQL_ACQUIRE="2", PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", SYSTEM_ACQUIRE_CHILD], env=env, cwd=root, capture_output=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-3000:]
    got = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert got["scope"] == 2, got
    assert got["aql_calls"] >= 300, got  # every call of the copy loop (the memset loop's wait for the null stream)
    assert got["bad"] == [], got
