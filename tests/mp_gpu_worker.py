"""One rank of the multi-process GPU collective tests (launched by
tests/test_gpu_collectives_mp.py; several ranks may share one GPU).
Runs every case of the spec through the MPI API and saves its result."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mvapich2_amd as m  # noqa: E402
from mvapich2_amd.consts import OPS, TYPES  # noqa: E402
from tests.helpers import rand_typed  # noqa: E402

WORLD = 0x44000000


def inputs(case, rank):
    rng = np.random.default_rng(case["seed"] * 1000 + rank)
    return rand_typed(case["type"], case["count"], rng, small=case.get("small", False))


def main():
    spec = json.load(open(sys.argv[1]))
    out = sys.argv[2]
    rank = int(os.environ["RANK"])
    n = int(os.environ["WORLD_SIZE"])
    L = m.lib()
    m.check(L.MPI_Init(None, None), "MPI_Init")
    L.MPI_Comm_set_errhandler(WORLD, 0x54000001)
    golden = None
    for case in spec["cases"]:
        k = case["kind"]
        t = case.get("type", "MPI_FLOAT")
        h, ext = TYPES[t][0], TYPES[t][3]
        count = case.get("count", 0)
        res = None
        if k in ("allreduce", "allreduce_inplace", "reduce", "iallreduce"):
            if "golden" in case:
                if golden is None:
                    golden = np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False)
                x = golden[case["golden"] + "__in"][rank]
            else:
                x = inputs(case, rank)
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(count * ext)
            rb.upload(np.full(count * ext, 0xA5, dtype=np.uint8))
            op = OPS[case["op"]]
            if k == "allreduce":
                rc = L.MPI_Allreduce(sb.ptr, rb.ptr, count, h, op, WORLD)
            elif k == "allreduce_inplace":
                rc = L.MPI_Allreduce(ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF), sb.ptr, count, h, op, WORLD)
                rb = sb
            elif k == "iallreduce":  # nonblocking: initiate, then MPI_Wait (completion word)
                req = ctypes.c_int()
                rc = L.MPI_Iallreduce(sb.ptr, rb.ptr, count, h, op, WORLD, ctypes.byref(req))
                if rc == 0:
                    rc = L.MPI_Wait(ctypes.byref(req), None)
            else:
                rc = L.MPI_Reduce(sb.ptr, rb.ptr, count, h, op, case["root"], WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=count * ext)
        elif k == "reduce_scatter":
            counts = case["recvcounts"]
            x = inputs(dict(case, count=sum(counts)), rank)
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(max(1, counts[rank]) * ext)
            arr = (ctypes.c_int * n)(*counts)
            rc = L.MPI_Reduce_scatter(sb.ptr, rb.ptr, arr, h, OPS[case["op"]], WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=counts[rank] * ext)
        elif k == "allgather":
            x = inputs(case, rank)
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(count * ext * n)
            rc = L.MPI_Allgather(sb.ptr, count, h, rb.ptr, count, h, WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=count * ext * n)
        elif k == "bcast":
            x = inputs(case, rank)
            b = m.DeviceBuffer.from_array(x)
            rc = L.MPI_Bcast(b.ptr, count, h, case["root"], WORLD)
            assert rc == 0, (case["id"], rc)
            res = b.download(np.uint8, count=count * ext)
        elif k == "user_allreduce":
            FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_int))

            def uop(inp, io, ln, dt):
                c = ln[0]
                a = np.ctypeslib.as_array((ctypes.c_int * c).from_address(inp))
                b = np.ctypeslib.as_array((ctypes.c_int * c).from_address(io))
                b[:] = a * 2 + b * 3
            cb = FN(uop)
            op = ctypes.c_int()
            L.MPI_Op_create(ctypes.cast(cb, ctypes.c_void_p), case["commute"], ctypes.byref(op))
            x = (np.arange(count, dtype=np.int32) + rank) % 7
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(count * 4)
            rc = L.MPI_Allreduce(sb.ptr, rb.ptr, count, TYPES["MPI_INT"][0], op.value, WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=count * 4)
            L.MPI_Op_free(ctypes.byref(op))
        elif k == "user_reduce_scatter":
            FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_int))

            def uop(inp, io, ln, dt):
                c = ln[0]
                a = np.ctypeslib.as_array((ctypes.c_int * c).from_address(inp))
                b = np.ctypeslib.as_array((ctypes.c_int * c).from_address(io))
                b[:] = a * 2 + b * 3
            cb = FN(uop)
            op = ctypes.c_int()
            L.MPI_Op_create(ctypes.cast(cb, ctypes.c_void_p), case["commute"], ctypes.byref(op))
            counts = case["recvcounts"]
            x = ((np.arange(sum(counts)) + rank) % 7).astype(np.int32)
            sb = m.DeviceBuffer.from_array(x)
            rb = m.DeviceBuffer(max(1, counts[rank]) * 4)
            arr = (ctypes.c_int * n)(*counts)
            rc = L.MPI_Reduce_scatter(sb.ptr, rb.ptr, arr, TYPES["MPI_INT"][0], op.value, WORLD)
            assert rc == 0, (case["id"], rc)
            res = rb.download(np.uint8, count=counts[rank] * 4)
            L.MPI_Op_free(ctypes.byref(op))
        elif k == "vector_bcast":
            # MPI_Type_vector(N, 4, 8, MPI_FLOAT) operand broadcast (device pack/unpack path)
            vt = ctypes.c_int()
            nb = case["nblocks"]
            assert L.MPI_Type_vector(nb, 4, 8, TYPES["MPI_FLOAT"][0], ctypes.byref(vt)) == 0
            assert L.MPI_Type_commit(ctypes.byref(vt)) == 0
            x = np.full(nb * 8, -1.0, dtype=np.float32)
            if rank == case["root"]:
                x = np.arange(nb * 8, dtype=np.float32)
            b = m.DeviceBuffer.from_array(x)
            rc = L.MPI_Bcast(b.ptr, 1, vt.value, case["root"], WORLD)
            assert rc == 0, (case["id"], rc)
            res = b.download(np.uint8, count=nb * 8 * 4)
            L.MPI_Type_free(ctypes.byref(vt))
        else:
            raise ValueError(k)
        np.save(os.path.join(out, f"{case['id']}_r{rank}.npy"), res)
    L.MPI_Finalize()
    print(f"rank {rank} done", flush=True)


if __name__ == "__main__":
    main()
