"""CPU: the multi-node allreduce table restatement of the library (orders.cpp mn_allreduce_table,
through mv2h_mn_allreduce_table) against the tests' own reading of the reference's table headers
(tests/test_gpu_multinode_mp.py table_entry: nemesis_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{2,1}ppn.h
numproc 2 / 4 / 8 entries, and the 16-ppn first entry through the oracle's one-node selection),
including each two-level entry's intra-node function (allreduce_osu.c:1727-1745)."""
import ctypes

import pytest

import mvapich2_amd as m
from oracle import oracle
from tests.test_gpu_multinode_mp import table_entry

FLAT = {2: "pt2pt_rs", 3: "pt2pt_rd"}
SIZES = sorted({1 << k for k in range(19)} | {(1 << k) + 1 for k in range(19)} | {(1 << k) - 1 for k in range(2, 19)}
               | {3000, 4800, 6000})


@pytest.mark.parametrize("ppn,gsize", [(1, 2), (1, 3), (1, 4), (1, 8), (2, 4), (2, 6), (2, 8), (3, 6), (4, 8),
                                       (3, 9), (4, 16)])
def test_table_matches_the_headers(ppn, gsize):
    L = m.lib()
    # the table itself: the small-message shortcuts (applied before the table, coll.cpp mn_select)
    # are off in the oracle's one-node reading of the 16-ppn entry
    k = oracle.default_knobs(enable_topo=0, enable_skip_search=0)
    for nbytes in SIZES:
        intra, inter = ctypes.c_int(), ctypes.c_int()
        t = L.mv2h_mn_allreduce_table(ppn, gsize, nbytes, ctypes.byref(intra), ctypes.byref(inter))
        kind, fn = table_entry(ppn, gsize, nbytes, knobs=k)
        tag = (ppn, gsize, nbytes, t, intra.value, inter.value, kind, fn)
        if kind == "flat":
            assert t in FLAT and FLAT[t] == fn, tag
            continue
        assert t == 0 and FLAT[inter.value] == fn, tag
        if ppn >= 3:
            assert intra.value == 0, tag  # the node's one-node selection reads the same 16-ppn entry
        else:
            idx = min(17, max(0, nbytes.bit_length() - 1))
            ci = (gsize // 2).bit_length() - 1
            assert intra.value == (3 if (ci == 2 and idx == 6) else 1), tag  # reduce_shmem (pt2pt_rs at one index)
