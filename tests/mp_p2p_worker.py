"""One rank of the multi-process point-to-point / nonblocking-collective GPU
tests (tests/test_gpu_p2p_mp.py; ranks may share one GPU).  Every check is
exact (byte patterns / integer sums) and asserted in the rank itself; a rank
exits non-zero on the first mismatch."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402

WORLD = 0x44000000
ANY_SOURCE, ANY_TAG, PROC_NULL = -2, -1, -1
INT, FLOAT, BYTE = TYPES["MPI_INT"][0], TYPES["MPI_FLOAT"][0], TYPES["MPI_BYTE"][0]


class Status(ctypes.Structure):
    _fields_ = [("count_lo", ctypes.c_int), ("count_hi_and_cancelled", ctypes.c_int), ("MPI_SOURCE", ctypes.c_int),
                ("MPI_TAG", ctypes.c_int), ("MPI_ERROR", ctypes.c_int)]


def pattern(nbytes, src, dst, tag):
    i = np.arange(nbytes, dtype=np.int64)
    return ((i * 131 + src * 7 + dst * 13 + tag * 29) % 251).astype(np.uint8)


def get_count(L, st, dt):
    c = ctypes.c_int()
    assert L.MPI_Get_count(ctypes.byref(st), dt, ctypes.byref(c)) == 0
    return c.value


def step(k):
    # where each rank was: a failed run prints every failed rank's tail (test_gpu_p2p_mp.py)
    print(f"rank {os.environ['RANK']} step {k}", flush=True)


def main():
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    L = m.lib()
    m.check(L.MPI_Init(None, None), "MPI_Init")
    L.MPI_Comm_set_errhandler(WORLD, 0x54000001)
    right, left = (rank + 1) % n, (rank - 1) % n

    step(1)
    # 1. ring exchange with Sendrecv at sizes below, at and above the 32 MiB channel ring (8 MiB chunks)
    for nbytes in (0, 1, 4093, 8 << 20, (8 << 20) + 17, 40 << 20):
        sb = m.DeviceBuffer.from_array(pattern(nbytes, rank, right, 5)) if nbytes else m.DeviceBuffer(1)
        rb = m.DeviceBuffer(max(nbytes, 1))
        st = Status()
        rc = L.MPI_Sendrecv(sb.ptr, nbytes, BYTE, right, 5, rb.ptr, nbytes, BYTE, left, 5, WORLD, ctypes.byref(st))
        assert rc == 0, ("sendrecv", nbytes, rc)
        assert st.MPI_SOURCE == left and st.MPI_TAG == 5 and get_count(L, st, BYTE) == nbytes, (st.MPI_SOURCE, st.MPI_TAG)
        if nbytes:
            got = rb.download(np.uint8, count=nbytes)
            assert np.array_equal(got, pattern(nbytes, left, rank, 5)), ("sendrecv data", nbytes)

    step(2)
    # 2. tag matching out of order + ANY_SOURCE/ANY_TAG: rank 0 receives from every
    #    other rank, tags posted in reverse of the send order (unexpected queue)
    if rank != 0:
        bufs = []
        for tag in (1, 2, 3):
            b = m.DeviceBuffer.from_array(pattern(3000 + tag, rank, 0, tag))
            bufs.append(b)
            assert L.MPI_Send(b.ptr, 3000 + tag, BYTE, 0, tag, WORLD) == 0
    else:
        for src in range(1, n):
            for tag in (3, 1, 2):
                rb = m.DeviceBuffer(4000)
                st = Status()
                assert L.MPI_Recv(rb.ptr, 4000, BYTE, src, tag, WORLD, ctypes.byref(st)) == 0
                assert st.MPI_TAG == tag and st.MPI_SOURCE == src and get_count(L, st, BYTE) == 3000 + tag
                assert np.array_equal(rb.download(np.uint8, count=3000 + tag), pattern(3000 + tag, src, 0, tag))
    L.MPI_Barrier(WORLD)
    if rank != 0:
        h = np.full(16, rank, dtype=np.int32)  # host buffer path
        assert L.MPI_Send(h.ctypes.data, 16, INT, 0, 100 + rank, WORLD) == 0
    else:
        seen = set()
        for _ in range(n - 1):
            h = np.zeros(16, dtype=np.int32)
            st = Status()
            assert L.MPI_Recv(h.ctypes.data, 16, INT, ANY_SOURCE, ANY_TAG, WORLD, ctypes.byref(st)) == 0
            assert st.MPI_TAG == 100 + st.MPI_SOURCE and np.all(h == st.MPI_SOURCE)
            seen.add(st.MPI_SOURCE)
        assert seen == set(range(1, n))

    step(3)
    # 3. Isend/Irecv both directions with Waitall (must not deadlock above the ring size)
    nbytes = 48 << 20
    sb = m.DeviceBuffer.from_array(pattern(nbytes, rank, right, 9))
    rb = m.DeviceBuffer(nbytes)
    q0, q1 = ctypes.c_int(), ctypes.c_int()
    assert L.MPI_Isend(sb.ptr, nbytes, BYTE, right, 9, WORLD, ctypes.byref(q0)) == 0
    assert L.MPI_Irecv(rb.ptr, nbytes, BYTE, left, 9, WORLD, ctypes.byref(q1)) == 0
    reqs = (ctypes.c_int * 2)(q0.value, q1.value)
    assert L.MPI_Waitall(2, reqs, None) == 0 and reqs[0] == reqs[1] == 0x2c000000
    assert np.array_equal(rb.download(np.uint8, count=nbytes), pattern(nbytes, left, rank, 9))

    step(4)
    # 4. truncation: 100 bytes into a 60-byte receive -> MPI_ERR_TRUNCATE (14), first 60 delivered
    sb = m.DeviceBuffer.from_array(pattern(100, rank, right, 11))
    rb = m.DeviceBuffer(60)
    rq = ctypes.c_int()
    assert L.MPI_Isend(sb.ptr, 100, BYTE, right, 11, WORLD, ctypes.byref(rq)) == 0
    rc = L.MPI_Recv(rb.ptr, 60, BYTE, left, 11, WORLD, None)
    assert rc == 14, rc
    assert np.array_equal(rb.download(np.uint8, count=60), pattern(100, left, rank, 11)[:60])
    assert L.MPI_Wait(ctypes.byref(rq), None) == 0

    step(5)
    # 5. MPI_PROC_NULL
    st = Status()
    assert L.MPI_Recv(rb.ptr, 60, BYTE, PROC_NULL, 0, WORLD, ctypes.byref(st)) == 0 and st.MPI_SOURCE == PROC_NULL

    step(6)
    # 6. derived type: MPI_Type_vector(64, 4, 8, MPI_FLOAT) send -> contiguous receive
    vt = ctypes.c_int()
    assert L.MPI_Type_vector(64, 4, 8, FLOAT, ctypes.byref(vt)) == 0 and L.MPI_Type_commit(ctypes.byref(vt)) == 0
    x = (np.arange(64 * 8, dtype=np.float32) + 1000 * rank)
    sb = m.DeviceBuffer.from_array(x)
    rb = m.DeviceBuffer(256 * 4)
    st = Status()
    assert L.MPI_Sendrecv(sb.ptr, 1, vt.value, right, 12, rb.ptr, 256, FLOAT, left, 12, WORLD, ctypes.byref(st)) == 0
    want = (np.arange(64 * 8, dtype=np.float32) + 1000 * left).reshape(64, 8)[:, :4].ravel()
    assert np.array_equal(rb.download(np.float32, count=256), want) and get_count(L, st, FLOAT) == 256
    L.MPI_Type_free(ctypes.byref(vt))

    step(7)
    # 7. nonblocking collectives: two Iallreduce in flight (pipelined + one-shot sizes), Ibcast, Wait/Test
    cnt = 3 << 20
    a = m.DeviceBuffer.from_array(np.arange(cnt, dtype=np.int32) * (rank + 1))
    ra = m.DeviceBuffer(cnt * 4)
    b = m.DeviceBuffer.from_array(np.full(1000, rank + 1, dtype=np.int32))
    rbb = m.DeviceBuffer(4000)
    c = m.DeviceBuffer.from_array(np.full(5000, 77 if rank == n - 1 else 0, dtype=np.int32))
    q = [ctypes.c_int() for _ in range(3)]
    assert L.MPI_Iallreduce(a.ptr, ra.ptr, cnt, INT, OPS["MPI_SUM"], WORLD, ctypes.byref(q[0])) == 0
    assert L.MPI_Iallreduce(b.ptr, rbb.ptr, 1000, INT, OPS["MPI_MAX"], WORLD, ctypes.byref(q[1])) == 0
    assert L.MPI_Ibcast(c.ptr, 5000, INT, n - 1, WORLD, ctypes.byref(q[2])) == 0
    flag = ctypes.c_int(0)
    while not flag.value:
        assert L.MPI_Test(ctypes.byref(q[0]), ctypes.byref(flag), None) == 0
    assert q[0].value == 0x2c000000
    r3 = (ctypes.c_int * 3)(*[x.value for x in q])
    assert L.MPI_Waitall(3, r3, None) == 0
    tri = n * (n + 1) // 2
    assert np.array_equal(ra.download(np.int32), (np.arange(cnt, dtype=np.int64) * tri).astype(np.int32))
    assert np.all(rbb.download(np.int32) == n)
    assert np.all(c.download(np.int32) == 77)
    step("7b")
    rq = ctypes.c_int()
    assert L.MPI_Ibarrier(WORLD, ctypes.byref(rq)) == 0 and L.MPI_Wait(ctypes.byref(rq), None) == 0

    step(8)
    # 8. MPI_Testall is all-or-nothing (MPI-3.1 §3.7.5): with one receive finished and one
    #    pending it returns flag = 0 and leaves both handles (and the finished one) intact
    if rank == 1:
        s20 = m.DeviceBuffer.from_array(pattern(777, 1, 0, 20))
        assert L.MPI_Send(s20.ptr, 777, BYTE, 0, 20, WORLD) == 0
        assert L.MPI_Recv(s20.ptr, 4, BYTE, 0, 22, WORLD, None) == 0  # rank 0's go-ahead
        s21 = m.DeviceBuffer.from_array(pattern(999, 1, 0, 21))
        assert L.MPI_Send(s21.ptr, 999, BYTE, 0, 21, WORLD) == 0
    elif rank == 0:
        import time
        r20, r21 = m.DeviceBuffer(777), m.DeviceBuffer(999)
        qa, qb = ctypes.c_int(), ctypes.c_int()
        assert L.MPI_Irecv(r20.ptr, 777, BYTE, 1, 20, WORLD, ctypes.byref(qa)) == 0
        assert L.MPI_Irecv(r21.ptr, 999, BYTE, 1, 21, WORLD, ctypes.byref(qb)) == 0
        pair = (ctypes.c_int * 2)(qa.value, qb.value)
        flag = ctypes.c_int(1)
        t_end = time.time() + 0.3
        while time.time() < t_end:  # the tag-20 message lands meanwhile; tag 21 cannot
            assert L.MPI_Testall(2, pair, ctypes.byref(flag), None) == 0
            assert flag.value == 0 and pair[0] == qa.value and pair[1] == qb.value, "Testall touched a request"
        one = (ctypes.c_int * 1)(qa.value)
        flag.value = 0
        while not flag.value:
            assert L.MPI_Testall(1, one, ctypes.byref(flag), None) == 0
        assert one[0] == 0x2c000000
        assert np.array_equal(r20.download(np.uint8, count=777), pattern(777, 1, 0, 20))
        go = m.DeviceBuffer(4)
        assert L.MPI_Send(go.ptr, 4, BYTE, 1, 22, WORLD) == 0
        rest = (ctypes.c_int * 1)(qb.value)
        flag.value = 0
        while not flag.value:
            assert L.MPI_Testall(1, rest, ctypes.byref(flag), None) == 0
        assert rest[0] == 0x2c000000
        assert np.array_equal(r21.download(np.uint8, count=999), pattern(999, 1, 0, 21))
    step(9)
    assert L.MPI_Barrier(WORLD) == 0
    assert L.MPI_Finalize() == 0
    print(f"rank {rank} p2p ok", flush=True)


if __name__ == "__main__":
    main()
