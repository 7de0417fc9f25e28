"""CPU: the multi-node allreduce table restatement of the library (orders.cpp mn_allreduce_table,
through mv2h_mn_allreduce_table) against the tests' reading of the reference's table headers
(tests/golden/mn_allreduce_tables.json, generated from
nemesis_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{1,2,16}ppn.h by tests/golden/gen_mn_allreduce_tables.py;
tests/test_gpu_multinode_mp.py table_cell), every numproc entry, including each two-level entry's
intra-node function (allreduce_osu.c:1727-1745)."""
import ctypes
import os
import json
from pathlib import Path

import pytest

import mvapich2_amd as m
from tests.test_gpu_multinode_mp import _TABLES, table_cell

FLAT = {2: "pt2pt_rs", 3: "pt2pt_rd"}
INTRA = {0: "node", 1: "reduce_shmem", 2: "reduce_p2p", 3: "pt2pt_rs", 4: "pt2pt_rd"}
SIZES = sorted({1 << k for k in range(19)} | {(1 << k) + 1 for k in range(19)} | {(1 << k) - 1 for k in range(2, 19)}
               | {3000, 4800, 6000, 1 << 22})
JOBS = [(1, 2), (1, 3), (1, 4), (1, 8), (1, 12), (1, 16), (1, 33), (1, 64), (1, 100), (2, 4), (2, 6), (2, 8), (2, 10),
        (2, 16), (2, 24), (2, 32), (2, 64), (3, 6), (4, 8), (3, 9), (4, 16), (3, 18), (4, 32), (8, 48), (8, 64),
        (16, 128), (16, 512), (16, 1024), (16, 4096)]


def test_fixture_covers_every_entry():
    # numproc lists of the three headers; 18 message-size indices per list
    assert [e["numproc"] for e in _TABLES["1ppn"]] == [2, 4, 8, 16, 32]
    assert [e["numproc"] for e in _TABLES["2ppn"]] == [2, 4, 8, 16, 32]
    assert [e["numproc"] for e in _TABLES["16ppn"]] == [16, 32, 64, 128, 256, 512, 1024]
    for tab in _TABLES.values():
        for e in tab:
            assert len(e["two_level"]) == len(e["inter"]) == len(e["intra"]) == 18, e


@pytest.mark.parametrize("ppn,gsize", JOBS)
def test_table_matches_the_headers(ppn, gsize):
    L = m.lib()
    for nbytes in SIZES:
        intra, inter = ctypes.c_int(), ctypes.c_int()
        t = L.mv2h_mn_allreduce_table(ppn, gsize, nbytes, ctypes.byref(intra), ctypes.byref(inter))
        kind, fn, want_intra = table_cell(ppn, gsize, nbytes)
        tag = (ppn, gsize, nbytes, t, intra.value, inter.value, kind, fn, want_intra)
        if kind == "flat":
            assert t in FLAT and FLAT[t] == fn, tag
            continue
        assert t == 0 and FLAT[inter.value] == fn and INTRA[intra.value] == want_intra, tag


# MPIR_Reduce_scatter_MV2's blocking table (tests/golden/red_scat_table.json, generated from
# red_scat_tuning.c by tests/golden/gen_red_scat_table.py) read as the reference reads it
# (red_scat_osu.c:1859-1893): the ring from the ring threshold; else the entry of the first
# numproc >= n (the last beyond); the first of its size_inter_table rows whose max >= nbytes
RS = json.loads((Path(__file__).parent / "golden" / "red_scat_table.json").read_text())
RS_CODE = {"rs_ring": 10, "rs_rec_halving": 11, "rs_pairwise": 12, "rs_basic": 13}


def rs_reference_choice(n, nbytes):
    if nbytes >= RS["ring_threshold"]:
        return "rs_ring"
    ents = RS["entries"]
    e = next((x for x in ents if n <= x["numproc"]), ents[-1])
    rt = 0
    while rt < e["size"] - 1 and nbytes > e["rows"][rt][1] and e["rows"][rt][1] != -1:
        rt += 1
    return e["rows"][rt][2]


@pytest.mark.parametrize("n", [2, 3, 8, 9, 12, 16, 17, 32, 33, 64, 65, 100, 128, 200, 512, 1000])
def test_reduce_scatter_table_matches_the_reference_table(n):
    L = m.lib()
    for nbytes in SIZES + [64, 65, 1024, 1025, 65536, 65537, 100000, 131071, 131072, 262144, 262145]:
        assert RS_CODE[rs_reference_choice(n, nbytes)] == L.mv2h_reduce_scatter_table(n, nbytes), (n, nbytes)


ROUTES = {0: "two-level", 1: "flat ring", 2: "flat programs", 3: "message schedule", 4: "two-level stand-in",
          5: "basic reduce-scatter"}
E_UNSUPPORTED = 44


@pytest.mark.parametrize("ppn,gsize", [(1, 2), (2, 8), (4, 12), (8, 16), (8, 64), (1, 65), (8, 72), (9, 72),
                                       (16, 128), (8, 128), (16, 1024)])
def test_every_builtin_route_is_supported(ppn, gsize):
    """above 64 ranks (no rank mesh) a flat algorithm's message schedule cannot
    run; the multi-node dispatch (coll.cpp mn_*_route) must then take the two-level stand-in, never
    refuse a builtin op.  Every size from 4 B to 1 GiB, blocking and nonblocking, IN_PLACE or not."""
    L = m.lib()
    rem = ctypes.c_int()
    for k in range(2, 31):
        for nbytes in (1 << k, (1 << k) + 4 * (gsize + 1)):
            count = nbytes // 4
            for coll, nbcs in ((0, (0, 1)), (1, (0, 2)), (2, (0, 3))):
                for nbc in nbcs:
                    for ip in (0, 1):
                        r = L.mv2h_mn_route(coll, ppn, gsize, nbytes, count, ip, nbc, ctypes.byref(rem))
                        where = (coll, nbytes, nbc, ip, r)
                        assert r in ROUTES and r != E_UNSUPPORTED, where
                        for route in (r, rem.value):
                            if route == 3:
                                assert 8 < gsize <= 64, where
                            if route == 2:
                                assert gsize <= 8, where
                            if route == 4:
                                assert gsize > 64, where
                        if coll == 2 and gsize > 64:
                            assert r == 5, where
    assert L.mv2h_mn_route(0, 3, 8, 64, 16, 0, 0, None) == 12  # 8 ranks are not 3 per node


RED_CODE = {"b": 7, "k": 8, "r": 9, "h": 1, "i": 8}


@pytest.mark.parametrize("cma", [1, 0])
def test_reduce_table_matches_the_headers(cma, monkeypatch):
    """orders.cpp mn_reduce_table (the multi-node MPI_Reduce selection, reduce_osu.c:2516-2620)
    against the tests' reading of tests/golden/mn_reduce_tables.json (generated from the reference's
    gen2{_cma}_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{1,2,16}ppn.h): every job shape, every size, the CMA
    and the plain tables (MV2_SMP_USE_CMA)"""
    from tests.test_gpu_multinode_mp import reduce_cell
    L = m.lib()
    monkeypatch.setenv("MV2_SMP_USE_CMA", str(cma))
    assert L.mv2h_knobs_reload() == 0
    try:
        tl, inter, intra, k = (ctypes.c_int() for _ in range(4))
        for ppn, gsize in JOBS + [(16, 32), (2, 4), (16, 48), (1, 3)]:
            for nbytes in SIZES + [1 << 19, 1 << 20, (1 << 21) + 5]:
                L.mv2h_mn_reduce_table(ppn, gsize, nbytes, ctypes.byref(tl), ctypes.byref(inter), ctypes.byref(intra),
                                       ctypes.byref(k))
                want = reduce_cell(ppn, gsize, nbytes, cma=bool(cma))
                assert (bool(tl.value), inter.value, intra.value, k.value) == \
                    (want[0], RED_CODE[want[1]], RED_CODE[want[2]], want[3]), (ppn, gsize, nbytes, cma)
    finally:
        monkeypatch.delenv("MV2_SMP_USE_CMA")
        L.mv2h_knobs_reload()


def test_reduce_table_reads_duplicate_first_entries_by_index():
    """the CMA 2- and 16-ppn tables list their first numproc twice; comm_size_index is arithmetic
    (reduce_osu.c:2537-2546), so 4 ranks at 2 ppn read the second "2" entry and 32 ranks at 16 ppn
    the second "16" entry, as the reference does"""
    L = m.lib()
    assert L.mv2h_mn_reduce_table(2, 4, 4096, None, None, None, None) == 1
    assert L.mv2h_mn_reduce_table(16, 32, 4096, None, None, None, None) == 1
    assert L.mv2h_mn_reduce_table(16, 64, 4096, None, None, None, None) == 2


def test_prog_max_knob_moves_flat_calls_onto_the_message_schedules():
    """MV2AMD_MN_PROG_MAX (coll.cpp mn_prog_max): with it at 4, an 8-rank job takes the message
    schedules that jobs above 8 ranks take, so the GPU tests cover them on 8 processes (DESIGN.md §5
    "Ranks per GPU"); unset, 8 ranks run as programs.  Read once per process: a child process."""
    import subprocess
    import sys
    code = ("import ctypes, mvapich2_amd as m; L = m.lib(); r = ctypes.c_int(); "
            "print(L.mv2h_mn_route(0, 4, 8, 64, 16, 0, 1, ctypes.byref(r)), "
            "L.mv2h_mn_route(0, 4, 8, 1 << 22, 1 << 20, 0, 0, ctypes.byref(r)), r.value)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    got = {}
    for v in (None, "4"):
        env = dict(os.environ)
        env.pop("MV2AMD_MN_PROG_MAX", None)
        if v:
            env["MV2AMD_MN_PROG_MAX"] = v
        out = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr
        got[v] = [int(x) for x in out.stdout.split()]
    # MPI_Iallreduce: flat over the job; 4 MiB allreduce: the ring with its remainder route
    assert got[None][0] == 2 and got["4"][0] == 3, got
    assert got[None][1] == got["4"][1], got
