#!/usr/bin/env python3
"""Generate the golden known-answer fixtures from the reference's own tests.

The reference (MVAPICH2 2.3.7) cannot be built in this image, so its
results are pinned through the known answers its MPICH test suite encodes.
This script restates, as data, the input patterns and expected outputs of:

  test/mpi/coll/allred.c       (every op x type group, np 4 and 7, count 10 / 100)
  test/mpi/coll/op{sum,prod,max,min,land,lor,lxor,band,bor,bxor,maxloc,minloc}.c
                               (3-element tie / identity patterns)
  test/mpi/coll/reduce_local.c (counts 0,1,2,4..32768; SUM on MPI_INT: 2i)
  test/mpi/coll/redscat.c      (sendbuf[i] = rank + i, recvcounts 1)

Expected values come from the formulas in those tests (C-type wraparound
reproduced with numpy fixed-width arithmetic), never from the oracle or the
HIP path.  Output: tests/golden/golden.npz + tests/golden/manifest.json.
Run: python tests/golden/make_golden.py
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# name -> (handle, numpy dtype)
SCALAR = {
    "MPI_INT": (0x4C000405, "i4"), "MPI_LONG": (0x4C000807, "i8"), "MPI_SHORT": (0x4C000203, "i2"),
    "MPI_UNSIGNED_SHORT": (0x4C000204, "u2"), "MPI_UNSIGNED": (0x4C000406, "u4"),
    "MPI_UNSIGNED_LONG": (0x4C000808, "u8"), "MPI_UNSIGNED_CHAR": (0x4C000102, "u1"),
    "MPI_INT8_T": (0x4C000137, "i1"), "MPI_INT16_T": (0x4C000238, "i2"), "MPI_INT32_T": (0x4C000439, "i4"),
    "MPI_INT64_T": (0x4C00083A, "i8"), "MPI_UINT8_T": (0x4C00013B, "u1"), "MPI_UINT16_T": (0x4C00023C, "u2"),
    "MPI_UINT32_T": (0x4C00043D, "u4"), "MPI_UINT64_T": (0x4C00083E, "u8"), "MPI_AINT": (0x4C000843, "i8"),
    "MPI_OFFSET": (0x4C000844, "i8"), "MPI_COUNT": (0x4C000845, "i8"),
    "MPI_FLOAT": (0x4C00040A, "f4"), "MPI_DOUBLE": (0x4C00080B, "f8"),
    "MPI_BYTE": (0x4C00010D, "u1"), "MPI_C_BOOL": (0x4C00013F, "u1"),
    "MPI_C_FLOAT_COMPLEX": (0x4C000840, "c8"), "MPI_C_DOUBLE_COMPLEX": (0x4C001041, "c16"),
    "MPI_CHAR": (0x4C000101, "i1"), "MPI_SIGNED_CHAR": (0x4C000118, "i1"),
}
PAIR = {
    "MPI_2INT": (0x4C000816, np.dtype([("a", "i4"), ("b", "i4")])),
    "MPI_LONG_INT": (0x8C000002, np.dtype({"names": ["a", "b"], "formats": ["i8", "i4"], "offsets": [0, 8], "itemsize": 16})),
    "MPI_SHORT_INT": (0x8C000003, np.dtype({"names": ["a", "b"], "formats": ["i2", "i4"], "offsets": [0, 4], "itemsize": 8})),
    "MPI_FLOAT_INT": (0x8C000000, np.dtype([("a", "f4"), ("b", "i4")])),
    "MPI_DOUBLE_INT": (0x8C000001, np.dtype({"names": ["a", "b"], "formats": ["f8", "i4"], "offsets": [0, 8], "itemsize": 16})),
}
OPS = {"MPI_MAX": 0x58000001, "MPI_MIN": 0x58000002, "MPI_SUM": 0x58000003, "MPI_PROD": 0x58000004,
       "MPI_LAND": 0x58000005, "MPI_BAND": 0x58000006, "MPI_LOR": 0x58000007, "MPI_BOR": 0x58000008,
       "MPI_LXOR": 0x58000009, "MPI_BXOR": 0x5800000A, "MPI_MINLOC": 0x5800000B, "MPI_MAXLOC": 0x5800000C}

# allred.c type sets (allred.c:285-330)
SET1 = ["MPI_INT", "MPI_LONG", "MPI_SHORT", "MPI_UNSIGNED_SHORT", "MPI_UNSIGNED", "MPI_UNSIGNED_LONG",
        "MPI_UNSIGNED_CHAR", "MPI_INT8_T", "MPI_INT16_T", "MPI_INT32_T", "MPI_INT64_T", "MPI_UINT8_T",
        "MPI_UINT16_T", "MPI_UINT32_T", "MPI_UINT64_T", "MPI_AINT", "MPI_OFFSET", "MPI_COUNT"]
SET2 = SET1 + ["MPI_FLOAT", "MPI_DOUBLE"]
SET3 = ["MPI_BYTE"]
SET4 = ["MPI_C_FLOAT_COMPLEX", "MPI_C_DOUBLE_COMPLEX"]
SET5 = ["MPI_C_BOOL"]

cases = []
arrays = {}


def add(family, tname, op, n, count, inputs, expected, fields=None, note=""):
    cid = f"{family}_{len(cases):04d}"
    arrays[cid + "__in"] = np.stack([np.ascontiguousarray(x).view(np.uint8).ravel() for x in inputs])
    arrays[cid + "__sol"] = np.ascontiguousarray(expected).view(np.uint8).ravel()
    handle = SCALAR[tname][0] if tname in SCALAR else PAIR[tname][0]
    cases.append({"id": cid, "family": family, "type": tname, "type_handle": handle, "op": op,
                  "op_handle": OPS[op], "n": n, "count": count, "fields": fields, "note": note})


def scalar_dtype(t):
    return np.dtype(SCALAR[t][1])


def cvt(vals, dt):
    """C assignment of int values into dt (wraps like the C conversion on x86-64)."""
    vals = np.asarray(vals, dtype=np.int64)
    if dt.kind in "iu":
        return vals.astype(np.uint64).astype(dt) if dt.kind == "u" else vals.astype(dt)
    return vals.astype(dt)


def allred_cases(n, count):
    i = np.arange(count)
    with np.errstate(over="ignore"):
        def scalar(test, tname, op, inp_fn, sol_fn):
            dt = scalar_dtype(tname)
            inputs = [inp_fn(r, dt) for r in range(n)]
            add("allred", tname, op, n, count, inputs, sol_fn(dt), note=f"allred.c {test}")

        for t in SET2:
            # sum_test1: in = i, sol = i*size (wrap in the C type)
            scalar("sum_test1", t, "MPI_SUM", lambda r, dt: cvt(i, dt), lambda dt: cvt(i * n, dt))
            # prod_test1: sol = i^size computed by repeated *= in the C type (SET_INDEX_POWER)
            def pw(dt):
                a = np.ones(count, dtype=dt)
                for _ in range(n):
                    a = (a * cvt(i, dt)).astype(dt)
                return a
            scalar("prod_test1", t, "MPI_PROD", lambda r, dt: cvt(i, dt), pw)
            scalar("max_test1", t, "MPI_MAX", lambda r, dt: cvt(i + r, dt), lambda dt: cvt(i + n - 1, dt))
            scalar("min_test1", t, "MPI_MIN", lambda r, dt: cvt(i + r, dt), lambda dt: cvt(i, dt))

        def const(test, tlist, op, v1, v2):
            for t in tlist:
                dt = scalar_dtype(t)
                inputs = [cvt(np.full(count, v1(r)), dt) for r in range(n)]
                add("allred", t, op, n, count, inputs, cvt(np.full(count, v2), dt), note=f"allred.c {test}")

        for tl in (SET1, SET5):
            const("lor_test1", tl, "MPI_LOR", lambda r: r & 1, int(n > 1))
            const("lor_test2", tl, "MPI_LOR", lambda r: 0, 0)
            const("lxor_test1", tl, "MPI_LXOR", lambda r: int(r == 1), int(n > 1))
            const("lxor_test2", tl, "MPI_LXOR", lambda r: 0, 0)
            const("lxor_test3", tl, "MPI_LXOR", lambda r: 1, n & 1)
            const("land_test1", tl, "MPI_LAND", lambda r: r & 1, 0)
            const("land_test2", tl, "MPI_LAND", lambda r: 1, 1)
        for tl in (SET1, SET3):
            const("bor_test1", tl, "MPI_BOR", lambda r: r & 3, (n - 1) if n < 3 else 3)
            const("bxor_test1", tl, "MPI_BXOR", lambda r: int(r == 1) * 0xF0, int(n > 1) * 0xF0)
            const("bxor_test2", tl, "MPI_BXOR", lambda r: 0, 0)
            const("bxor_test3", tl, "MPI_BXOR", lambda r: -1, -1 if (n & 1) else 0)
            for t in tl:
                dt = scalar_dtype(t)
                ins = [cvt(i, dt) if r == n - 1 else cvt(np.full(count, -1), dt) for r in range(n)]
                add("allred", t, "MPI_BAND", n, count, ins, cvt(i, dt), note="allred.c band_test1")
                ins = [cvt(i, dt) if r == n - 1 else cvt(np.zeros(count), dt) for r in range(n)]
                add("allred", t, "MPI_BAND", n, count, ins, cvt(np.zeros(count), dt), note="allred.c band_test2")
        for t in SET4:
            dt = scalar_dtype(t)
            add("allred", t, "MPI_SUM", n, count, [i.astype(dt) for _ in range(n)], (i * n).astype(dt),
                note="allred.c sum_test1 (complex)")
            sol = np.ones(count, dtype=dt)
            for _ in range(n):
                sol = sol * i.astype(dt)
            add("allred", t, "MPI_PROD", n, count, [i.astype(dt) for _ in range(n)], sol,
                note="allred.c prod_test1 (complex)")
        for t, (h, dt) in PAIR.items():
            for op in ("MPI_MAXLOC", "MPI_MINLOC"):
                ins = []
                for r in range(n):
                    x = np.zeros(count, dtype=dt)
                    x["a"] = (i + r).astype(dt["a"])
                    x["b"] = r
                    ins.append(x)
                sol = np.zeros(count, dtype=dt)
                if op == "MPI_MAXLOC":
                    sol["a"] = (i + n - 1).astype(dt["a"])
                    sol["b"] = n - 1
                else:
                    sol["a"] = i.astype(dt["a"])
                    sol["b"] = 0
                add("allred", t, op, n, count, ins, sol, fields=["a", "b"], note=f"allred.c {op.lower()}_test")


def op3_cases(n):
    """3-element patterns of test/mpi/coll/op*.c (rank 0 result)."""
    maxsize = min(n, 5)
    fact = [1, 1, 2, 6, 24, 120]
    types_int = ["MPI_CHAR", "MPI_SIGNED_CHAR", "MPI_UNSIGNED_CHAR", "MPI_SHORT", "MPI_UNSIGNED_SHORT",
                 "MPI_INT", "MPI_UNSIGNED", "MPI_LONG", "MPI_UNSIGNED_LONG"]
    types_fp = ["MPI_FLOAT", "MPI_DOUBLE"]
    pats = {
        "MPI_SUM": (types_int + types_fp, lambda r: [1, 0, int(r > 0)], [n, 0, n - 1], "opsum.c"),
        "MPI_PROD": (types_int + types_fp, lambda r: [r if (0 < r < maxsize) else 1, 0, int(r > 1)],
                     [fact[maxsize - 1], 0, 0 if n > 1 else 0], "opprod.c"),
        "MPI_MAX": (types_int + types_fp, lambda r: [1, 0, r], [1, 0, n - 1], "opmax.c"),
        "MPI_MIN": (types_int + types_fp, lambda r: [1, 0, r & 0x7F], [1, 0, 0], "opmin.c"),
        "MPI_LAND": (types_int + types_fp, lambda r: [1, 0, int(r > 0)], [1, 0, 0], "opland.c"),
        "MPI_LOR": (types_int + types_fp, lambda r: [1, 0, int(r > 0)], [1, 0, int(n > 1)], "oplor.c"),
        "MPI_LXOR": (types_int + types_fp, lambda r: [1, 0, int(r > 0)], [n % 2, 0, (n - 1) % 2], "oplxor.c"),
        "MPI_BAND": (types_int, lambda r: [0xFF, 0, 0xFF if r > 0 else 0xF0], [0xFF, 0, 0xF0], "opband.c"),
        "MPI_BOR": (types_int, lambda r: [0xFF, 0, 0x3C if r > 0 else 0xC3], [0xFF, 0, 0xFF if n > 1 else 0xC3], "opbor.c"),
        "MPI_BXOR": (types_int, lambda r: [0xFF, 0, 0x3C if r > 0 else 0xC3],
                     [0xFF if n % 2 else 0, 0, 0xC3 if n % 2 else 0xFF], "opbxor.c"),
    }
    for op, (tl, inp, sol, src) in pats.items():
        for t in tl:
            dt = scalar_dtype(t)
            ins = [cvt(inp(r), dt) for r in range(n)]
            add("op3", t, op, n, 3, ins, cvt(sol, dt), note=src)
    # opmaxloc.c / opminloc.c: ties resolve to the minimum location
    for t, (h, dt) in PAIR.items():
        ins = []
        for r in range(n):
            x = np.zeros(3, dtype=dt)
            x["a"] = np.array([1, 0, r], dtype=dt["a"])
            x["b"] = r
            ins.append(x)
        sol = np.zeros(3, dtype=dt)
        sol["a"] = np.array([1, 0, n - 1], dtype=dt["a"])
        sol["b"] = [0, 0, n - 1]
        add("op3", t, "MPI_MAXLOC", n, 3, ins, sol, fields=["a", "b"], note="opmaxloc.c")
        ins = []
        for r in range(n):
            x = np.zeros(3, dtype=dt)
            x["a"] = np.array([1, 0, r & 0x7F], dtype=dt["a"])
            x["b"] = r
            ins.append(x)
        sol = np.zeros(3, dtype=dt)
        sol["a"] = np.array([1, 0, 0], dtype=dt["a"])
        sol["b"] = [0, 0, 0]
        add("op3", t, "MPI_MINLOC", n, 3, ins, sol, fields=["a", "b"], note="opminloc.c")


def reduce_local_cases():
    count = 0
    while count < 65000:
        i = np.arange(count, dtype=np.int32)
        add("reduce_local", "MPI_INT", "MPI_SUM", 2, count, [i, i], 2 * i, note="reduce_local.c (in, inout)")
        count = count * 2 if count > 0 else 1


def redscat_cases(n):
    for r in range(1):
        pass
    ins = [np.array([r + i for i in range(n)], dtype=np.int32) for r in range(n)]
    sol = np.array([(n * (r + (r + n - 1))) // 2 for r in range(n)], dtype=np.int32)
    add("redscat", "MPI_INT", "MPI_SUM", n, n, ins, sol, note="redscat.c recvcounts[i] = 1")


def main():
    for n, count in ((4, 10), (7, 10), (4, 100)):
        allred_cases(n, count)
    for n in (4, 7):
        op3_cases(n)
    reduce_local_cases()
    for n in (4, 6):
        redscat_cases(n)
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"source": "restated known answers of MVAPICH2 2.3.7 test/mpi/coll tests",
                   "generator": "tests/golden/make_golden.py", "cases": cases}, f, indent=0)
    print(f"{len(cases)} cases written")


if __name__ == "__main__":
    main()
