"""The drop-in boundary: libmpi.so loads without a GPU and exports every
symbol include/*.h declares (MPI_* as weak aliases of PMPI_*), and its
host-side tables (datatype sizes, op x type legality) equal the oracle's."""
import ctypes
import os
import re
import subprocess

import pytest

import mvapich2_amd as m
from mvapich2_amd.consts import OPS, TYPES
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"^\s*(?:int|double|const char \*)\s*((?:P?MPIX?|mv2h)_\w+)\(", txt, flags=re.M))


def exported():
    out = subprocess.run(["nm", "-D", "--defined-only", m.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) == 3:
            syms[parts[2]] = parts[1]
    return syms


def test_library_loads_without_gpu():
    L = m.lib()
    assert b"gfx950" in L.mv2h_version()


@pytest.mark.parametrize("header", ["mpi.h", "mv2h.h"])
def test_every_declared_symbol_is_exported(header):
    syms = exported()
    names = declared(header)
    assert len(names) > 20
    missing = sorted(n for n in names if n not in syms)
    assert not missing, missing


def test_mpi_symbols_are_weak_aliases_of_pmpi():
    syms = exported()
    for n in declared("mpi.h"):
        if n.startswith("MPI_") or n.startswith("MPIX_"):
            assert syms.get(n) == "W", n
            assert syms.get("P" + n) == "T", n


def test_soname_is_mpich_abi():
    out = subprocess.run(["readelf", "-d", m.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "libmpi.so.12" in out


def test_dtype_table_matches_oracle():
    L = m.lib()
    for t, (h, desc, size, ext) in TYPES.items():
        s, e = ctypes.c_size_t(), ctypes.c_size_t()
        assert L.mv2h_dtype_info(h, ctypes.byref(s), ctypes.byref(e)) == 0, t
        os_, oe = ctypes.c_long(), ctypes.c_long()
        assert oracle.lib().oracle_dtype_info(h, ctypes.byref(os_), ctypes.byref(oe)) == 0
        assert (s.value, e.value) == (size, ext) == (os_.value, oe.value), t


def test_op_legality_matches_oracle():
    L = m.lib()
    for op, oh in OPS.items():
        for t, (h, *_r) in TYPES.items():
            assert (L.mv2h_op_check(oh, h) == 0) == (oracle.op_check(oh, h) == 0), (op, t)
    assert L.mv2h_op_check(OPS["MPI_SUM"], 0x12345) == 3  # unknown type -> MPI_ERR_TYPE


def test_op_table_header_symbols_are_exported():
    """include/mpir_op.h: the predefined ops as MPI_User_function entry points
    (MPIR_Op_table, allreduce.c:95-107) — every declared name and both tables."""
    txt = open(os.path.join(ROOT, "include", "mpir_op.h")).read()
    names = set(re.findall(r"^\s*(?:void|int)\s+(MPIR_\w+)\(", txt, flags=re.M))
    assert len(names) == 29
    syms = exported()
    missing = sorted(n for n in names | {"MPIR_Op_table", "MPIR_Op_check_dtype_table"} if n not in syms)
    assert not missing, missing


def test_op_table_check_dtype_matches_legality():
    """MPIR_OP_HDL_TO_DTYPE_FN(op)(type) == MPI_SUCCESS exactly where the op accepts the type
    (host-side tables only: no GPU call)."""
    L = m.lib()
    table = (ctypes.c_void_p * 14).in_dll(L, "MPIR_Op_check_dtype_table")
    CHK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int)
    for op, oh in OPS.items():
        fn = CHK(table[(oh & 0xF) - 1])
        for t, (h, *_r) in TYPES.items():
            want = 0 if L.mv2h_op_check(oh, h) == 0 else 9  # MPI_ERR_OP
            assert fn(h) == want, (op, t)
        assert fn(0x1234) == 3  # not a datatype: MPI_ERR_TYPE


def test_collops_plugin_symbols_and_attach_without_world():
    """include/mv2amd_collops.h (MPID_Collops members, mpiimpl.h:1999-2033): every entry is
    exported; a communicator that is not the node world is refused with MPI_ERR_COMM and every
    entry then returns MPI_ERR_COMM before touching data (the caller falls back)."""
    txt = open(os.path.join(ROOT, "include", "mv2amd_collops.h")).read()
    names = set(re.findall(r"^\s*int\s+(MV2AMD_\w+)\(", txt, flags=re.M))
    assert len(names) == 10
    syms = exported()
    assert not sorted(n for n in names if n not in syms)
    L = m.lib()
    fake = ctypes.c_void_p(0x1000)
    assert L.MV2AMD_Comm_attach(fake, 0, 99) == 5  # MPI_ERR_COMM: not this world's size
    err = ctypes.c_int(0)
    assert L.MV2AMD_Allreduce(None, None, 4, TYPES["MPI_FLOAT"][0], OPS["MPI_SUM"], fake, ctypes.byref(err)) == 5
    assert L.MV2AMD_Barrier(fake, ctypes.byref(err)) == 5
    assert err.value == 0
    ops = (ctypes.c_void_p * 7)()
    assert L.MV2AMD_Collops_get(ops) == 0
    assert all(ops)
