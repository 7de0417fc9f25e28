"""MPI_T tool interface (mpi/mpit.cpp): the hot path's per-algorithm counters and
timers under the reference's names and categories (src/mpi_t/mv2_mpit.c), and the
MV2_* selection knobs as control variables.  Host-side only: no GPU call (the GPU
multiprocess test checks the counts collectives produce)."""
import ctypes

import pytest

import mvapich2_amd as m

T_ERR_NOT_INITIALIZED, T_ERR_INVALID_INDEX, T_ERR_INVALID_NAME = 60, 62, 73
T_ERR_CVAR_SET_NEVER, T_ERR_PVAR_NO_WRITE = 69, 71
CLASS_COUNTER, CLASS_TIMER = 246, 248
MPI_UNSIGNED_LONG_LONG, MPI_DOUBLE = 0x4C000819, 0x4C00080B

EXPECTED_COUNTERS = [
    "mv2_coll_allreduce_shm_rd", "mv2_coll_allreduce_shm_rs", "mv2_coll_allreduce_shm_intra",
    "mv2_coll_allreduce_intra_p2p", "mv2_coll_allreduce_2lvl", "mv2_coll_allreduce_topo_aware_hierarchical",
    "mv2_coll_allreduce_pt2pt_ring", "mv2_coll_allreduce_pt2pt_ring_wrapper", "mv2_coll_allreduce_pt2pt_ring_inplace",
    "mv2_coll_reduce_binomial", "mv2_coll_reduce_redscat_gather", "mv2_coll_reduce_shmem", "mv2_coll_reduce_knomial",
    "mv2_coll_reduce_topo_aware_hierarchical", "mv2_coll_reduce_two_level_helper", "mv2_coll_reduce_scatter_basic",
    "mv2_coll_reduce_scatter_rec_halving", "mv2_coll_reduce_scatter_pairwise", "mv2_coll_reduce_scatter_ring",
    "mv2_coll_reduce_scatter_ring_2lvl", "mv2_coll_reduce_scatter_non_comm", "mv2_coll_reduce_scatter_noncomm",
    "mv2_num_shmem_coll_calls"]


@pytest.fixture
def T():
    L = m.lib()
    prov = ctypes.c_int()
    assert L.MPI_T_init_thread(3, ctypes.byref(prov)) == 0
    yield L
    assert L.MPI_T_finalize() == 0


def info(L, i):
    name, desc = ctypes.create_string_buffer(256), ctypes.create_string_buffer(512)
    nl, dl = ctypes.c_int(256), ctypes.c_int(512)
    verb, cls, dt, en, bind, ro, cont, at = (ctypes.c_int() for _ in range(8))
    assert L.MPI_T_pvar_get_info(i, name, ctypes.byref(nl), ctypes.byref(verb), ctypes.byref(cls), ctypes.byref(dt),
                                 ctypes.byref(en), desc, ctypes.byref(dl), ctypes.byref(bind), ctypes.byref(ro),
                                 ctypes.byref(cont), ctypes.byref(at)) == 0
    return dict(name=name.value.decode(), nl=nl.value, cls=cls.value, dt=dt.value & 0xFFFFFFFF, ro=ro.value,
                cont=cont.value, bind=bind.value, verb=verb.value)


def test_not_initialized_is_an_error():
    n = ctypes.c_int()
    assert m.lib().MPI_T_pvar_get_num(ctypes.byref(n)) == T_ERR_NOT_INITIALIZED


def test_pvar_names_classes_and_types(T):
    n = ctypes.c_int()
    assert T.MPI_T_pvar_get_num(ctypes.byref(n)) == 0
    infos = [info(T, i) for i in range(n.value)]
    counters = [x["name"] for x in infos if x["cls"] == CLASS_COUNTER]
    timers = [x["name"] for x in infos if x["cls"] == CLASS_TIMER]
    assert counters == EXPECTED_COUNTERS
    assert len(timers) == len(EXPECTED_COUNTERS) - 1  # mv2_num_shmem_coll_calls has no timer
    assert all(t.startswith("mv2_coll_timer_") for t in timers)
    for x in infos:
        assert x["nl"] == len(x["name"]) + 1
        assert x["ro"] == 1 and x["cont"] == 0 and x["bind"] == 9700 and x["verb"] == 221
        assert x["dt"] == (MPI_UNSIGNED_LONG_LONG if x["cls"] == CLASS_COUNTER else MPI_DOUBLE)
    idx = ctypes.c_int()
    assert T.MPI_T_pvar_get_index(b"mv2_coll_allreduce_shm_rs", CLASS_COUNTER, ctypes.byref(idx)) == 0
    assert infos[idx.value]["name"] == "mv2_coll_allreduce_shm_rs"
    assert T.MPI_T_pvar_get_index(b"mv2_coll_allreduce_shm_rs", CLASS_TIMER, ctypes.byref(idx)) == T_ERR_INVALID_NAME
    assert T.MPI_T_pvar_get_info(n.value, None, None, None, None, None, None, None, None, None, None, None,
                                 None) == T_ERR_INVALID_INDEX


def test_name_length_convention(T):
    """MPI-3.1 14.3.3: a short buffer gets len-1 characters and NUL; the length returned is strlen+1."""
    buf, nl = ctypes.create_string_buffer(8), ctypes.c_int(8)
    z = ctypes.c_int()
    assert T.MPI_T_pvar_get_info(0, buf, ctypes.byref(nl), None, ctypes.byref(z), None, None, None, None, None,
                                 None, None, None) == 0
    assert buf.value == b"mv2_col" and nl.value == len("mv2_coll_allreduce_shm_rd") + 1


def test_categories(T):
    n = ctypes.c_int()
    assert T.MPI_T_category_get_num(ctypes.byref(n)) == 0
    names = []
    for c in range(n.value):
        name, nl = ctypes.create_string_buffer(64), ctypes.c_int(64)
        nc, npv, ncat = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert T.MPI_T_category_get_info(c, name, ctypes.byref(nl), None, None, ctypes.byref(nc), ctypes.byref(npv),
                                         ctypes.byref(ncat)) == 0
        names.append((name.value.decode(), nc.value, npv.value))
    assert names[0] == ("Allreduce Algorithms", 0, 18)
    assert names[1] == ("Reduce Algorithms", 0, 12)
    assert names[2] == ("Reduce_scatter Algorithms", 0, 14)
    assert names[3] == ("Shmem Collective Calls", 0, 1)
    assert names[4][0] == "Collective Selection" and names[4][1] > 20
    idx = (ctypes.c_int * 18)()
    assert T.MPI_T_category_get_pvars(0, 18, idx) == 0
    assert info(T, idx[0])["name"] == "mv2_coll_allreduce_shm_rd"


def test_session_handles_start_stop_read_and_readonly(T):
    s = ctypes.c_void_p()
    assert T.MPI_T_pvar_session_create(ctypes.byref(s)) == 0
    i = ctypes.c_int()
    assert T.MPI_T_pvar_get_index(b"mv2_coll_allreduce_shm_rs", CLASS_COUNTER, ctypes.byref(i)) == 0
    h, cnt = ctypes.c_void_p(), ctypes.c_int()
    assert T.MPI_T_pvar_handle_alloc(s, i.value, None, ctypes.byref(h), ctypes.byref(cnt)) == 0 and cnt.value == 1
    all_h = ctypes.c_void_p.in_dll(T, "MPI_T_PVAR_ALL_HANDLES")
    assert T.MPI_T_pvar_start(s, all_h) == 0
    v = ctypes.c_ulonglong(99)
    assert T.MPI_T_pvar_read(s, h, ctypes.byref(v)) == 0 and v.value == 0
    assert T.MPI_T_pvar_stop(s, h) == 0
    assert T.MPI_T_pvar_write(s, h, ctypes.byref(v)) == T_ERR_PVAR_NO_WRITE
    assert T.MPI_T_pvar_reset(s, h) == T_ERR_PVAR_NO_WRITE
    assert T.MPI_T_pvar_handle_free(s, ctypes.byref(h)) == 0 and not h.value
    assert T.MPI_T_pvar_session_free(ctypes.byref(s)) == 0 and not s.value


def test_cvars_are_the_selection_knobs(T, monkeypatch):
    monkeypatch.setenv("MV2_ALLREDUCE_RING_ALGO_THRESHOLD", "64K")
    monkeypatch.setenv("MV2_SHMEM_REDUCE_TREE_DEGREE", "2")
    T.mv2h_knobs_reload()
    try:
        for name, want, nbytes in ((b"MV2_ALLREDUCE_RING_ALGO_THRESHOLD", 65536, 8),
                                   (b"MV2_SHMEM_REDUCE_TREE_DEGREE", 2, 4), (b"MV2_RED_SCAT_RING_ALGO_THRESHOLD", 131072, 8),
                                   (b"MV2_TOPO_AWARE_ALLREDUCE_MAX_MSG", 2048, 4)):
            i = ctypes.c_int()
            assert T.MPI_T_cvar_get_index(name, ctypes.byref(i)) == 0
            h, cnt = ctypes.c_void_p(), ctypes.c_int()
            assert T.MPI_T_cvar_handle_alloc(i.value, None, ctypes.byref(h), ctypes.byref(cnt)) == 0
            v = (ctypes.c_longlong if nbytes == 8 else ctypes.c_int)()
            assert T.MPI_T_cvar_read(h, ctypes.byref(v)) == 0
            assert v.value == want, name
            assert T.MPI_T_cvar_write(h, ctypes.byref(v)) == T_ERR_CVAR_SET_NEVER
            assert T.MPI_T_cvar_handle_free(ctypes.byref(h)) == 0
    finally:
        monkeypatch.delenv("MV2_ALLREDUCE_RING_ALGO_THRESHOLD")
        monkeypatch.delenv("MV2_SHMEM_REDUCE_TREE_DEGREE")
        T.mv2h_knobs_reload()
