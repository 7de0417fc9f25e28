"""mvapich2_amd — MI355X-native device-buffer reduction / collective hot path
of MVAPICH2 2.3.7, exported as an MPICH-ABI ``libmpi.so`` (include/mpi.h)
over a HIP C-ABI (include/mv2h.h).

This module is a thin ctypes binding used by the tests and bench.py.  It
loads the in-tree ``mvapich2_amd/lib/libmpi.so`` and fails loudly if that
library (the HIP path) is missing: there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

from . import consts
from .consts import OPS, TYPES

_HERE = os.path.dirname(os.path.abspath(__file__))
# MV2AMD_LIBMPI: another build of the same library (the host-sanitizer build the CPU tests can run)
LIB_PATH = os.environ.get("MV2AMD_LIBMPI") or os.path.join(_HERE, "lib", "libmpi.so")
_lib = None


class MPIError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what} failed with MPI error class {code}")
        self.code = code


def lib():
    """Load libmpi.so (built by __graft_entry__.build / make -C mvapich2_amd/csrc)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP library missing: {LIB_PATH} (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    c_vp, c_sz, c_int = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    sigs = {
        "mv2h_version": ([], ctypes.c_char_p),
        "mv2h_device_count": ([], c_int),
        "mv2h_is_device_ptr": ([c_vp], c_int),
        "mv2h_malloc": ([ctypes.POINTER(c_vp), c_sz], c_int),
        "mv2h_free": ([c_vp], c_int),
        "mv2h_memcpy_htod": ([c_vp, c_vp, c_sz], c_int),
        "mv2h_memcpy_dtoh": ([c_vp, c_vp, c_sz], c_int),
        "mv2h_memcpy_dtod": ([c_vp, c_vp, c_sz], c_int),
        "mv2h_memset": ([c_vp, c_int, c_sz], c_int),
        "mv2h_device_synchronize": ([], c_int),
        "mv2h_dtype_info": ([c_int, ctypes.POINTER(c_sz), ctypes.POINTER(c_sz)], c_int),
        "mv2h_op_check": ([c_int, c_int], c_int),
        "mv2h_reduce_local": ([c_vp, c_vp, c_sz, c_int, c_int, c_vp], c_int),
        "mv2h_reduce_n": ([ctypes.POINTER(c_vp), c_int, c_vp, c_sz, c_int, c_int, c_int, c_int, c_vp], c_int),
        "mv2h_allreduce": ([c_vp, c_vp, c_sz, c_int, c_int, c_vp], c_int),
        "mv2h_reduce": ([c_vp, c_vp, c_sz, c_int, c_int, c_int, c_vp], c_int),
        "mv2h_reduce_scatter": ([c_vp, c_vp, ctypes.POINTER(c_sz), c_int, c_int, c_vp], c_int),
        "mv2h_allgather": ([c_vp, c_vp, c_sz, c_vp], c_int),
        "mv2h_bcast": ([c_vp, c_sz, c_int, c_vp], c_int),
        "mv2h_barrier": ([], c_int),
        "mv2h_pack_strided": ([c_vp, c_vp, c_sz, c_sz, c_sz, c_vp], c_int),
        "mv2h_unpack_strided": ([c_vp, c_vp, c_sz, c_sz, c_sz, c_vp], c_int),
        "mv2h_pack_segments": ([c_vp, c_vp, c_sz, c_sz, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                c_int, c_int, c_vp], c_int),
        "mv2h_init": ([], c_int),
        "mv2h_finalize": ([], c_int),
        "mv2h_rank": ([], c_int),
        "mv2h_size": ([], c_int),
        "mv2h_local_rank": ([], c_int),
        "mv2h_timing_enable": ([c_int], c_int),
        "mv2h_last_kernel_ms": ([], ctypes.c_double),
        "mv2h_set_tuning": ([ctypes.c_char_p, ctypes.c_long], c_int),
        "mv2h_plan": ([c_int, c_int, c_int, c_int, c_sz, ctypes.POINTER(c_sz), c_int, c_int, c_int,
                       ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_vp], c_int),
        "mv2h_knobs_reload": ([], c_int),
        "mv2h_mn_allreduce_table": ([c_int, c_int, ctypes.c_long, ctypes.POINTER(c_int), ctypes.POINTER(c_int)], c_int),
        "mv2h_reduce_scatter_table": ([c_int, ctypes.c_long], c_int),
        "mv2h_rs_noncomm_expr": ([c_int, c_int, c_int] + [ctypes.POINTER(c_int)] * 3 + [c_int, ctypes.POINTER(c_int)], c_int),
        "mv2h_host_sched_eval": ([c_int] * 7 + [ctypes.c_void_p, ctypes.c_void_p], c_int),
        "mv2h_mn_reduce_table": ([c_int, c_int, ctypes.c_long] + [ctypes.POINTER(c_int)] * 4, c_int),
        "mv2h_mn_route": ([c_int, c_int, c_int, ctypes.c_long, ctypes.c_size_t, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "mv2h_nbc_begin": ([c_int], c_int),
        "mv2h_nbc_end": ([], c_int),
        "mv2h_get_info": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_long)], c_int),
        "mv2h_reduce_n_prog": ([ctypes.POINTER(c_vp), c_int, c_vp, c_sz, c_int, c_int, c_vp, c_vp], c_int),
        "MPI_Init": ([c_vp, c_vp], c_int),
        "MPI_Finalize": ([], c_int),
        "MPI_Comm_rank": ([c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Comm_size": ([c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Barrier": ([c_int], c_int),
        "MPI_Wtime": ([], ctypes.c_double),
        "MPI_Comm_set_errhandler": ([c_int, c_int], c_int),
        "MPI_Reduce_local": ([c_vp, c_vp, c_int, c_int, c_int], c_int),
        "MPI_Allreduce": ([c_vp, c_vp, c_int, c_int, c_int, c_int], c_int),
        "MPI_Reduce": ([c_vp, c_vp, c_int, c_int, c_int, c_int, c_int], c_int),
        "MPI_Reduce_scatter": ([c_vp, c_vp, ctypes.POINTER(c_int), c_int, c_int, c_int], c_int),
        "MPI_Reduce_scatter_block": ([c_vp, c_vp, c_int, c_int, c_int, c_int], c_int),
        "MPI_Allgather": ([c_vp, c_int, c_int, c_vp, c_int, c_int, c_int], c_int),
        "MPI_Bcast": ([c_vp, c_int, c_int, c_int, c_int], c_int),
        "MPI_Op_create": ([c_vp, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Op_free": ([ctypes.POINTER(c_int)], c_int),
        "MPI_Type_vector": ([c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Type_contiguous": ([c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Type_create_hvector": ([c_int, c_int, ctypes.c_long, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Type_create_indexed_block": ([c_int, c_int, ctypes.POINTER(c_int), c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Type_create_hindexed_block": ([c_int, c_int, ctypes.POINTER(ctypes.c_long), c_int,
                                            ctypes.POINTER(c_int)], c_int),
        "MPI_Type_indexed": ([c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Type_create_hindexed": ([c_int, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_long), c_int,
                                      ctypes.POINTER(c_int)], c_int),
        "MPI_Type_create_struct": ([c_int, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_long), ctypes.POINTER(c_int),
                                    ctypes.POINTER(c_int)], c_int),
        "MPI_Type_create_resized": ([c_int, ctypes.c_long, ctypes.c_long, ctypes.POINTER(c_int)], c_int),
        "MPI_Type_dup": ([c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Type_create_subarray": ([c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_int,
                                      c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Type_get_true_extent": ([c_int, ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_long)], c_int),
        "MPI_Type_commit": ([ctypes.POINTER(c_int)], c_int),
        "MPI_Type_free": ([ctypes.POINTER(c_int)], c_int),
        "MPI_Type_size": ([c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Type_get_extent": ([c_int, ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_long)], c_int),
        "MPI_Pack": ([c_vp, c_int, c_int, c_vp, c_int, ctypes.POINTER(c_int), c_int], c_int),
        "MPI_Unpack": ([c_vp, c_int, ctypes.POINTER(c_int), c_vp, c_int, c_int, c_int], c_int),
        "MPI_Pack_size": ([c_int, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        # nonblocking collectives / requests / point-to-point
        "MPI_Iallreduce": ([c_vp, c_vp, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Ireduce": ([c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Ireduce_scatter_block": ([c_vp, c_vp, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Iallgather": ([c_vp, c_int, c_int, c_vp, c_int, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Ibcast": ([c_vp, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Ibarrier": ([c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Wait": ([ctypes.POINTER(c_int), c_vp], c_int),
        "MPI_Test": ([ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_vp], c_int),
        "MPI_Waitall": ([c_int, ctypes.POINTER(c_int), c_vp], c_int),
        "MPI_Send": ([c_vp, c_int, c_int, c_int, c_int, c_int], c_int),
        "MPI_Recv": ([c_vp, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "MPI_Isend": ([c_vp, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Irecv": ([c_vp, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)], c_int),
        "MPI_Sendrecv": ([c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "MPI_Get_count": ([c_vp, c_int, ctypes.POINTER(c_int)], c_int),
        # stream-ordered collectives (extension; the last argument is a hipStream_t)
        "MPIX_Allreduce_enqueue": ([c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp], c_int),
        "MPIX_Reduce_enqueue": ([c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp], c_int),
        "MPIX_Reduce_scatter_enqueue": ([c_vp, c_vp, ctypes.POINTER(c_int), c_int, c_int, c_int, c_vp], c_int),
        "MPIX_Allgather_enqueue": ([c_vp, c_int, c_int, c_vp, c_int, c_int, c_int, c_vp], c_int),
        "MPIX_Bcast_enqueue": ([c_vp, c_int, c_int, c_int, c_int, c_vp], c_int),
        "MPIX_Enqueue_check": ([c_int], c_int),
    }
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        raise MPIError(rc, what)


def np_dtype(type_name):
    desc = TYPES[type_name][1]
    if desc == "f16":
        return np.dtype(np.longdouble)
    return np.dtype(desc)


class DeviceBuffer:
    """A hipMalloc'd buffer owned by the library's allocator."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(lib().mv2h_malloc(ctypes.byref(p), max(self.nbytes, 1)), "mv2h_malloc")
        self.ptr = p.value

    @classmethod
    def from_array(cls, arr):
        arr = np.ascontiguousarray(arr)
        b = cls(arr.nbytes)
        b.upload(arr)
        return b

    def upload(self, arr, offset=0):
        arr = np.ascontiguousarray(arr)
        if arr.nbytes:
            check(lib().mv2h_memcpy_htod(self.ptr + offset, arr.ctypes.data, arr.nbytes), "htod")

    def download(self, dtype, count=None, offset=0):
        dt = np.dtype(dtype)
        n = (self.nbytes - offset) // dt.itemsize if count is None else count
        out = np.empty(n, dtype=dt)
        if out.nbytes:
            check(lib().mv2h_memcpy_dtoh(out.ctypes.data, self.ptr + offset, out.nbytes), "dtoh")
        return out

    def free(self):
        if self.ptr:
            lib().mv2h_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def reduce_local(inbuf, inoutbuf, count, type_name, op_name, offset_in=0, offset_io=0):
    """MPI_Reduce_local on device buffers through the C-ABI (mv2h_reduce_local)."""
    return lib().mv2h_reduce_local(inbuf.ptr + offset_in, inoutbuf.ptr + offset_io, count,
                                   TYPES[type_name][0], OPS[op_name], None)


__all__ = ["lib", "check", "DeviceBuffer", "MPIError", "reduce_local", "np_dtype", "consts", "OPS", "TYPES"]


# ---- reduction-order plans (host only) ----
class Prog(ctypes.Structure):
    _fields_ = [("nsteps", ctypes.c_uint8), ("res", ctypes.c_uint8), ("dst", ctypes.c_uint8 * 7),
                ("src", ctypes.c_uint8 * 7)]


class ProgSet(ctypes.Structure):
    _fields_ = [("nprog", ctypes.c_int32), ("pad", ctypes.c_int32), ("blk", ctypes.c_uint64), ("p", Prog * 8)]


COLL = {"allreduce": 0, "reduce": 1, "reduce_scatter": 2, "allreduce_rs": 3}


def plan(coll, n, rank, dtype_handle, count=0, counts=None, root=0, opkind=0, in_place=False):
    """(algo, inner, unpinned, programs, blk): the algorithm MVAPICH2 picks for this call
    and its per-block reduction programs [(steps[(dst, src)...], res), ...]."""
    L = lib()
    algo, inner, unp = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    ps = ProgSet()
    cz = (ctypes.c_size_t * n)(*counts) if counts is not None else None
    check(L.mv2h_plan(COLL[coll], n, rank, root, count, cz, dtype_handle, opkind, int(in_place), ctypes.byref(algo),
                      ctypes.byref(inner), ctypes.byref(unp), ctypes.byref(ps)), "mv2h_plan")
    progs = [([(p.dst[i], p.src[i]) for i in range(p.nsteps)], p.res) for p in ps.p[:ps.nprog]]
    return algo.value, inner.value, unp.value, progs, ps.blk


NBC = {"iallreduce": 1, "ireduce": 2, "ireduce_scatter": 3, "reduce_scatter_block": 4}


class nbc:
    """Context: plan() / the reducing collectives take the nonblocking selection `kind`
    (or MPI_Reduce_scatter_block's) on this thread (mv2h_nbc_begin / mv2h_nbc_end)."""

    def __init__(self, kind):
        self.kind = NBC[kind]

    def __enter__(self):
        check(lib().mv2h_nbc_begin(self.kind), "mv2h_nbc_begin")
        return self

    def __exit__(self, *exc):
        lib().mv2h_nbc_end()
        return False


def knobs_reload():
    check(lib().mv2h_knobs_reload(), "mv2h_knobs_reload")


def info(key):
    v = ctypes.c_long()
    check(lib().mv2h_get_info(key.encode(), ctypes.byref(v)), f"mv2h_get_info({key})")
    return v.value
