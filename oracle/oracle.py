"""ctypes loader for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / the timed CPU baseline.  The product
(mvapich2_amd) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH) or os.path.getmtime(_PATH) < os.path.getmtime(os.path.join(_HERE, "mv2_oracle.c")):
            build()
        L = ctypes.CDLL(_PATH)
        vp, l, i = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
        L.oracle_reduce_local.argtypes = [vp, vp, l, i, i]
        L.oracle_op_check.argtypes = [i, i]
        L.oracle_dtype_info.argtypes = [i, ctypes.POINTER(l), ctypes.POINTER(l)]
        L.oracle_allreduce.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), i, l, i, i, i]
        L.oracle_allreduce_algo.argtypes = [i, l, i]
        L.oracle_reduce_linear.argtypes = [ctypes.POINTER(vp), i, vp, l, i, i]
        L.oracle_reduce_scatter_ring.argtypes = [ctypes.POINTER(vp), i, ctypes.POINTER(l), vp, i, i]
        L.oracle_pack_strided.argtypes = [vp, vp, l, l, l]
        L.oracle_pack_strided.restype = None
        L.oracle_unpack_strided.argtypes = [vp, vp, l, l, l]
        L.oracle_unpack_strided.restype = None
        L.oracle_pack_segments.argtypes = [vp, vp, l, l, ctypes.POINTER(l), ctypes.POINTER(l), i, i]
        L.oracle_pack_segments.restype = None
        L.oracle_time_reduce_local.argtypes = [vp, vp, l, i, i, i]
        L.oracle_time_reduce_local.restype = ctypes.c_double
        _lib = L
    return _lib


def reduce_local(inp, inout, count, dtype_handle, op_handle):
    """inout <- op(inout, inp) in place on numpy arrays; returns the rc."""
    return lib().oracle_reduce_local(inp.ctypes.data, inout.ctypes.data, count, dtype_handle, op_handle)


def op_check(op_handle, dtype_handle):
    return lib().oracle_op_check(op_handle, dtype_handle)


def allreduce(sends, count, dtype_handle, op_handle, algo=-1):
    """Simulate MV2 MPI_Allreduce over len(sends) ranks; returns per-rank results."""
    n = len(sends)
    recvs = [np.zeros_like(s) for s in sends]
    sp = (ctypes.c_void_p * n)(*[s.ctypes.data for s in sends])
    rp = (ctypes.c_void_p * n)(*[r.ctypes.data for r in recvs])
    rc = lib().oracle_allreduce(sp, rp, n, count, dtype_handle, op_handle, algo)
    if rc:
        raise RuntimeError(f"oracle_allreduce rc={rc}")
    return recvs


def reduce_linear(srcs, count, dtype_handle, op_handle):
    n = len(srcs)
    dst = np.zeros_like(srcs[0])
    sp = (ctypes.c_void_p * n)(*[s.ctypes.data for s in srcs])
    rc = lib().oracle_reduce_linear(sp, n, dst.ctypes.data, count, dtype_handle, op_handle)
    if rc:
        raise RuntimeError(f"oracle_reduce_linear rc={rc}")
    return dst


def reduce_scatter_ring(srcs, counts, dtype_handle, op_handle):
    """Every block of MPIR_Reduce_scatter_ring's result (red_scat_osu.c:1026-1180), concatenated."""
    n = len(srcs)
    dst = np.zeros_like(srcs[0])
    sp = (ctypes.c_void_p * n)(*[s.ctypes.data for s in srcs])
    cn = (ctypes.c_long * n)(*counts)
    rc = lib().oracle_reduce_scatter_ring(sp, n, cn, dst.ctypes.data, dtype_handle, op_handle)
    if rc:
        raise RuntimeError(f"oracle_reduce_scatter_ring rc={rc}")
    return dst


def pack_strided(src, nblocks, blk, stride):
    dst = np.zeros(nblocks * blk, dtype=np.uint8)
    lib().oracle_pack_strided(src.ctypes.data, dst.ctypes.data, nblocks, blk, stride)
    return dst


def pack_segments(src, dst, count, extent, offs, lens, unpack=False):
    """Segment-walk pack (unpack=False: src strided -> dst packed) or unpack."""
    n = len(offs)
    lo = (ctypes.c_long * n)(*offs)
    ll = (ctypes.c_long * n)(*lens)
    lib().oracle_pack_segments(src.ctypes.data, dst.ctypes.data, count, extent, lo, ll, n, 1 if unpack else 0)
    return dst


def unpack_strided(packed, dst, nblocks, blk, stride):
    lib().oracle_unpack_strided(packed.ctypes.data, dst.ctypes.data, nblocks, blk, stride)
    return dst
