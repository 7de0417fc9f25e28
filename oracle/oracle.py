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


class Knobs(ctypes.Structure):
    """MV2_* selection knobs (oknobs in mv2_oracle.c); default_knobs() = the reference defaults."""
    _fields_ = [(f, ctypes.c_int) for f in (
        "coll_skip_thr", "enable_skip_search", "allred_skip_small", "allred_skip_large",
        "enable_topo", "use_topo_allreduce", "topo_allred_min", "topo_allred_max",
        "use_topo_reduce", "topo_red_min", "topo_red_max", "tree_degree",
        "allred_use_ring", "ring_ppn")] + [("ring_thr", ctypes.c_long), ("red_scat_ring_thr", ctypes.c_long)] + [
        (f, ctypes.c_int) for f in ("smp_use_cma", "inter_k", "use_knomial_reduce", "shmem_intra_reduce_msg",
                                    "shmem_coll_max_msg", "enable_shmem_allreduce", "enable_shmem_reduce")]


# algorithm ids (include/mv2h.h mv2h_plan)
ALGOS = ["none", "shmem_linear", "pt2pt_rs", "pt2pt_rd", "ring_wrapper", "topo_tree", "two_level_p2p",
         "binomial", "knomial", "redscat_gather", "rs_ring", "rs_rec_halving", "rs_pairwise", "rs_basic",
         "reduce_topo", "rs_noncomm_pof2", "rs_noncomm_rd"]


def default_knobs(**over):
    k = Knobs()
    lib().oracle_default_knobs(ctypes.byref(k))
    for key, v in over.items():
        setattr(k, key, v)
    return k


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
        kp = ctypes.POINTER(Knobs)
        L.oracle_default_knobs.argtypes = [kp]
        L.oracle_default_knobs.restype = None
        L.oracle_allreduce_select.argtypes = [i, l, i, i, i, kp]
        L.oracle_allreduce_k.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), i, l, i, i, i, kp]
        L.oracle_reduce_select.argtypes = [i, l, i, i, kp, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.oracle_reduce.argtypes = [ctypes.POINTER(vp), vp, i, l, i, i, i, i, kp, i]
        L.oracle_reduce_scatter_select.argtypes = [i, ctypes.POINTER(l), i, kp]
        L.oracle_reduce_scatter.argtypes = [ctypes.POINTER(vp), i, ctypes.POINTER(l), vp, i, i, kp, i]
        L.oracle_iallreduce_select.argtypes = [i, l, i, i, l]
        L.oracle_reduce_scatter_block_select.argtypes = [i, l, i, l]
        L.oracle_set_topology.argtypes = [i, ctypes.POINTER(i), i]
        L.oracle_set_topology.restype = None
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


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def allreduce_select(n, count, dtype_handle, in_place=False, opkind=0, knobs=None):
    k = knobs if knobs is not None else default_knobs()
    return lib().oracle_allreduce_select(n, count, dtype_handle, int(in_place), opkind, ctypes.byref(k))


def allreduce_ref(sends, count, dtype_handle, op_handle, in_place=False, knobs=None):
    """MPI_Allreduce as MVAPICH2 2.3.7 runs it on one node (selection + algorithm), per-rank results."""
    n = len(sends)
    k = knobs if knobs is not None else default_knobs()
    recvs = [np.zeros_like(s) for s in sends]
    rc = lib().oracle_allreduce_k(_ptrs(sends), _ptrs(recvs), n, count, dtype_handle, op_handle, int(in_place),
                                  ctypes.byref(k))
    if rc:
        raise RuntimeError(f"oracle_allreduce_k rc={rc}")
    return recvs


def reduce_select(n, count, dtype_handle, opkind=0, knobs=None):
    k = knobs if knobs is not None else default_knobs()
    kf, r0 = ctypes.c_int(0), ctypes.c_int(0)
    a = lib().oracle_reduce_select(n, count, dtype_handle, opkind, ctypes.byref(k), ctypes.byref(kf), ctypes.byref(r0))
    return a, kf.value, r0.value


def reduce_ref(sends, count, dtype_handle, op_handle, root, opkind=0, knobs=None, algo=-1):
    """MPI_Reduce as MVAPICH2 2.3.7 runs it on one node: the root's result."""
    k = knobs if knobs is not None else default_knobs()
    out = np.zeros_like(sends[0])
    rc = lib().oracle_reduce(_ptrs(sends), out.ctypes.data, len(sends), count, dtype_handle, op_handle, root, opkind,
                             ctypes.byref(k), algo)
    if rc:
        raise RuntimeError(f"oracle_reduce rc={rc}")
    return out


def reduce_scatter_select(counts, dtype_handle, knobs=None):
    k = knobs if knobs is not None else default_knobs()
    n = len(counts)
    return lib().oracle_reduce_scatter_select(n, (ctypes.c_long * n)(*counts), dtype_handle, ctypes.byref(k))


def reduce_scatter_ref(srcs, counts, dtype_handle, op_handle, knobs=None, algo=-1):
    """MPI_Reduce_scatter as MVAPICH2 2.3.7 runs it on one node: every rank's block, concatenated."""
    k = knobs if knobs is not None else default_knobs()
    n = len(srcs)
    dst = np.zeros_like(srcs[0])
    rc = lib().oracle_reduce_scatter(_ptrs(srcs), n, (ctypes.c_long * n)(*counts), dst.ctypes.data, dtype_handle,
                                     op_handle, ctypes.byref(k), algo)
    if rc:
        raise RuntimeError(f"oracle_reduce_scatter rc={rc}")
    return dst


def iallreduce_select(n, count, dtype_handle, opkind=0, short_msg=2048):
    """MPI_Iallreduce on one node: naive = Ireduce to rank 0 (binomial or redscat_gather) + Ibcast"""
    return lib().oracle_iallreduce_select(n, count, dtype_handle, opkind, short_msg)


def iallreduce_ref(sends, count, dtype_handle, op_handle, opkind=0, short_msg=2048):
    """every rank's MPI_Iallreduce result: rank 0's Ireduce result"""
    a = iallreduce_select(len(sends), count, dtype_handle, opkind, short_msg)
    r0 = reduce_ref(sends, count, dtype_handle, op_handle, 0, opkind=opkind, algo=a)
    return [r0.copy() for _ in sends]


def ireduce_ref(sends, count, dtype_handle, op_handle, root, opkind=0):
    """MPI_Ireduce on one node: MPIR_Ireduce_binomial"""
    return reduce_ref(sends, count, dtype_handle, op_handle, root, opkind=opkind, algo=ALGOS.index("binomial"))


def reduce_scatter_block_select(n, recvcount, dtype_handle, long_msg=524288):
    return lib().oracle_reduce_scatter_block_select(n, recvcount, dtype_handle, long_msg)


def set_topology(levels, n):
    """Intra-node topology of the topology-aware shm tree: levels = [[cluster id of rank r at level l
    for r < n] for each level l] (the NUMA node, then the socket); [] = one group."""
    flat = [c for lv in levels for c in lv]
    lib().oracle_set_topology(len(levels), (ctypes.c_int * max(1, len(flat)))(*flat), n)
