// coll.cpp — the mv2h_* C-ABI (include/mv2h.h): op layer entry points and
// host orchestration of the device collectives.
//
// Algorithm / order selection restates the reference's single-node choice
// (generic table allreduce_tuning.c:2734-2750, selection allreduce_osu.c:
// 3146-3375): nbytes < 1024 -> two-level reduce_shmem order (LINEAR),
// otherwise pt2pt_rs order (BUTTERFLY; recursive-doubling owner when
// count < pof2, allreduce_osu.c:802).  The data path is MI355X-native:
// one-shot push through uncached IPC arenas for small messages, direct
// reduce-scatter + all-gather over xGMI peer mappings for large ones.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>

#include "../../../include/mv2h.h"
#include "log.h"
#include "world.h"

namespace mv2 {

int log_rank() { return world().rank; }
bool log_debug_on() {
    static int on = -1;
    if (on < 0) {
        const char *v = getenv("MV2AMD_DEBUG");
        on = (v && *v && *v != '0') ? 1 : 0;
    }
    return on == 1;
}

static hipStream_t pick_stream(void *s) { return s ? (hipStream_t)s : world().stream; }

static int finish(hipStream_t st, bool timed) {
    World &w = world();
    if (hipStreamSynchronize(st) != hipSuccess) {
        MV2_ERR("hipStreamSynchronize failed: %s", hipGetErrorString(hipGetLastError()));
        return E_INTERN;
    }
    if (timed) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, w.ev0, w.ev1);
        w.last_ms = ms;
    }
    if (w.h_err && __atomic_load_n(w.h_err, __ATOMIC_ACQUIRE)) {
        MV2_ERR("device collective timed out waiting for a peer (MV2AMD_TIMEOUT_S)");
        __atomic_store_n(w.h_err, 0, __ATOMIC_RELEASE);
        return E_OTHER;
    }
    return 0;
}

static inline void tmark0(hipStream_t st) {
    if (world().timing) hipEventRecord(world().ev0, st);
}
static inline void tmark1(hipStream_t st) {
    if (world().timing) hipEventRecord(world().ev1, st);
}

// 1 = device memory (hipMalloc / IPC-importable), 0 = anything else
static int is_device(const void *p) {
    if (!p) return 0;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        hipGetLastError();
        return 0;
    }
    return a.type == hipMemoryTypeDevice ? 1 : 0;
}

static int kind_supported(const DtypeInfo *dt) {
    if (!dt) return E_TYPE;
    if (dt->kind == K_LDOUBLE) {
        MV2_ERR("%s: x87 80-bit long double has no gfx950 representation (not supported on device)", dt->name);
        return E_TYPE;
    }
    return 0;
}

static int check_op_dtype(int op, int dtype, const DtypeInfo **out) {
    const DtypeInfo *dt = dtype_lookup(dtype);
    if (!dt) return E_TYPE;
    if (!is_builtin_op(op)) return E_OP;
    if (!op_valid_for_groups(op_index(op), dt->groups)) return E_OP;
    *out = dt;
    return 0;
}

// ---------------------------------------------------------------------------
// reduction order
// ---------------------------------------------------------------------------
static TreeParams make_tree(int n, size_t count, const DtypeInfo *dt, int me) {
    TreeParams tp{};
    int pof2 = 1, lg = 0;
    while (pof2 * 2 <= n) { pof2 *= 2; ++lg; }
    tp.pof2 = pof2;
    tp.lg = lg;
    tp.rem = n - pof2;
    tp.linear = (count * (size_t)dt->size < 1024) ? 1 : 0;
    tp.owner_fixed = 0;
    tp.rs_blk = 0;
    if (!tp.linear) {
        if (count >= (size_t)pof2) {
            tp.owner_fixed = -1;
            tp.rs_blk = count / pof2;
        } else {
            // recursive doubling: each rank keeps its own result; even ranks
            // below 2*rem receive their odd partner's (allreduce_osu.c:585-600)
            int r = me;
            if (r < 2 * tp.rem && r % 2 == 0) r = r + 1;
            tp.owner_fixed = (r < 2 * tp.rem) ? r / 2 : r - tp.rem;
        }
    }
    return tp;
}

static int grid_cap() {
    World &w = world();
    int g = w.max_grid / (w.nshare > 0 ? w.nshare : 1);
    if (g < 1) g = 1;
    if (g > kMaxBlocks) g = kMaxBlocks;
    return g;
}

// launch config of a collective kernel: identical on every rank (the grid
// must match across ranks: workgroup b of each rank pairs with workgroup b)
static LaunchCfg coll_cfg(int grid, hipStream_t st) {
    World &w = world();
    LaunchCfg c{grid, 2, st};
    c.cus = w.cus;
    c.nshare = w.nshare;
    return c;
}

// ---------------------------------------------------------------------------
// IPC export / import of user buffers
// ---------------------------------------------------------------------------
static int publish(int slot, const void *ptr) {
    World &w = world();
    BufDesc &d = w.shm->r[w.rank].desc[slot];
    uint64_t bid = 0;
    hipDeviceptr_t base = nullptr;
    size_t asz = 0;
    if (hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)ptr) != hipSuccess ||
        hipMemGetAddressRange(&base, &asz, (hipDeviceptr_t)ptr) != hipSuccess) {
        hipGetLastError();
        MV2_ERR("buffer %p is not a device allocation that can be shared over IPC", ptr);
        return E_BUFFER;
    }
    auto it = w.own_handles.find(bid);
    if (it == w.own_handles.end()) {
        hipIpcMemHandle_t h;
        if (hipIpcGetMemHandle(&h, (void *)base) != hipSuccess) {
            hipGetLastError();
            MV2_ERR("hipIpcGetMemHandle failed for %p", ptr);
            return E_BUFFER;
        }
        it = w.own_handles.emplace(bid, h).first;
    }
    d.handle = it->second;
    d.buffer_id = bid;
    d.base = (uint64_t)(uintptr_t)base;
    d.alloc_size = asz;
    d.offset = (uint64_t)((const char *)ptr - (const char *)base);
    d.seq = w.seq;
    return 0;
}

// pointer of peer j's published buffer `slot` in this process
static const char *peer_buffer(int j, int slot, int *rc) {
    World &w = world();
    const BufDesc &d = w.shm->r[j].desc[slot];
    if (d.seq != w.seq) {
        MV2_ERR("rank %d published a stale buffer descriptor (seq %llu vs %llu)", j,
                (unsigned long long)d.seq, (unsigned long long)w.seq);
        *rc = E_INTERN;
        return nullptr;
    }
    auto &m = w.peer_maps[j];
    auto it = m.find(d.buffer_id);
    if (it == m.end()) {
        // a cached mapping whose peer range overlaps this new allocation belongs to
        // a buffer the peer has freed (its address was reused): unmap it
        for (auto e = m.begin(); e != m.end();) {
            const Mapping &mp = e->second;
            if (mp.peer_base < d.base + d.alloc_size && d.base < mp.peer_base + mp.alloc_size) {
                hipIpcCloseMemHandle(mp.ptr);
                e = m.erase(e);
                continue;
            }
            ++e;
        }
        if (m.size() >= 64) {
            auto victim = std::min_element(m.begin(), m.end(), [](const auto &a, const auto &b) {
                return a.second.last_use < b.second.last_use;
            });
            hipIpcCloseMemHandle(victim->second.ptr);
            m.erase(victim);
        }
        void *p = nullptr;
        if (hipIpcOpenMemHandle(&p, d.handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            hipGetLastError();
            MV2_ERR("hipIpcOpenMemHandle failed for rank %d buffer", j);
            *rc = E_OTHER;
            return nullptr;
        }
        it = m.emplace(d.buffer_id, Mapping{(char *)p, d.base, d.alloc_size, 0}).first;
    }
    it->second.last_use = ++w.use_clock;
    *rc = 0;
    return it->second.ptr + d.offset;
}

}  // namespace mv2

using namespace mv2;

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

const char *mv2h_version(void) { return "mvapich2_amd 0.1 (MI355X gfx950; MVAPICH2 2.3.7 device-buffer hot path)"; }

int mv2h_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int mv2h_is_device_ptr(const void *p) { return is_device(p); }

int mv2h_malloc(void **p, size_t bytes) {
    if (ensure_init_for_device()) return E_OTHER;
    return hipMalloc(p, bytes ? bytes : 1) == hipSuccess ? 0 : E_NO_MEM;
}
int mv2h_free(void *p) { return hipFree(p) == hipSuccess ? 0 : E_ARG; }
int mv2h_memcpy_htod(void *d, const void *s, size_t b) { return hipMemcpy(d, s, b, hipMemcpyHostToDevice) == hipSuccess ? 0 : E_INTERN; }
int mv2h_memcpy_dtoh(void *d, const void *s, size_t b) { return hipMemcpy(d, s, b, hipMemcpyDeviceToHost) == hipSuccess ? 0 : E_INTERN; }
int mv2h_memcpy_dtod(void *d, const void *s, size_t b) { return hipMemcpy(d, s, b, hipMemcpyDeviceToDevice) == hipSuccess ? 0 : E_INTERN; }
int mv2h_memset(void *d, int v, size_t b) { return hipMemset(d, v, b) == hipSuccess ? 0 : E_INTERN; }
int mv2h_device_synchronize(void) { return hipDeviceSynchronize() == hipSuccess ? 0 : E_INTERN; }

int mv2h_dtype_info(int dtype, size_t *size, size_t *extent) {
    const DtypeInfo *dt = dtype_lookup(dtype);
    if (!dt) return E_TYPE;
    if (size) *size = dt->size;
    if (extent) *extent = dt->extent;
    return 0;
}

int mv2h_op_check(int op, int dtype) {
    const DtypeInfo *dt = nullptr;
    return check_op_dtype(op, dtype, &dt);
}

int mv2h_timing_enable(int on) {
    world().timing = on != 0;
    return 0;
}
double mv2h_last_kernel_ms(void) { return world().last_ms; }

int mv2h_set_tuning(const char *key, long value) {
    World &w = world();
    if (!strcmp(key, "max_grid")) w.max_grid = (int)value;
    else if (!strcmp(key, "rl_grid")) w.rl_grid = (int)value;
    else if (!strcmp(key, "oneshot_max")) {
        if ((size_t)value > w.slot_bytes && w.size > 1) return E_ARG;
        w.oneshot_max = (size_t)value;
    } else return E_ARG;
    return 0;
}

int mv2h_init(void) { return world_init(); }
int mv2h_finalize(void) { return world_finalize(); }
int mv2h_rank(void) { return world().rank; }
int mv2h_size(void) { return world().size; }
int mv2h_local_rank(void) { return world().local_rank; }

int mv2h_barrier(void) {
    host_barrier();
    return 0;
}

// ---------------------------------------------------------------------------
// part (1): MPI_Reduce_local on device buffers (reduce_local.c:36-173)
// ---------------------------------------------------------------------------
int mv2h_reduce_local(const void *in, void *inout, size_t count, int dtype, int op, void *stream) {
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    if (count == 0) return 0;  // reduce_local.c:49
    if ((rc = kind_supported(dt))) return rc;
    if ((rc = ensure_init_for_device())) return rc;
    World &w = world();
    hipStream_t st = pick_stream(stream);
    const int oi = op_index(op);
    const size_t bytes = count * (size_t)dt->extent;
    // host buffers: staged through device scratch, reduced on the GPU
    const bool din = is_device(in), dio = is_device(inout);
    const void *din_p = in;
    void *dio_p = inout;
    if (!din) {
        void *s = get_scratch(0, bytes);
        if (!s) return E_NO_MEM;
        hipMemcpyAsync(s, in, bytes, hipMemcpyHostToDevice, st);
        din_p = s;
    }
    if (!dio) {
        void *s = get_scratch(1, bytes);
        if (!s) return E_NO_MEM;
        hipMemcpyAsync(s, inout, bytes, hipMemcpyHostToDevice, st);
        dio_p = s;
    }
    tmark0(st);
    if (oi == OP_NO_OP) {
        rc = 0;
    } else if (oi == OP_REPLACE) {
        rc = hipMemcpyAsync(dio_p, din_p, bytes, hipMemcpyDeviceToDevice, st) == hipSuccess ? 0 : E_INTERN;
    } else {
        LaunchCfg cfg{w.rl_grid, 4, st};
        rc = launch_reduce_local(oi, dt->kind, din_p, dio_p, count, dt->extent, cfg);
    }
    tmark1(st);
    if (rc) return rc;
    if (!dio) hipMemcpyAsync(inout, dio_p, bytes, hipMemcpyDeviceToHost, st);
    return finish(st, w.timing);
}

int mv2h_reduce_n(const void *const *srcs, int nsrc, void *dst, size_t count, int dtype, int op, int order,
                  int owner, void *stream) {
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    if ((rc = kind_supported(dt))) return rc;
    if (nsrc < 1 || nsrc > kMaxRanks) return E_ARG;
    if (count == 0) return 0;
    if ((rc = ensure_init_for_device())) return rc;
    const int oi = op_index(op);
    if (oi >= OP_REPLACE) return E_OP;
    hipStream_t st = pick_stream(stream);
    TreeParams tp{};
    int pof2 = 1, lg = 0;
    while (pof2 * 2 <= nsrc) { pof2 *= 2; ++lg; }
    tp.pof2 = pof2;
    tp.lg = lg;
    tp.rem = nsrc - pof2;
    tp.linear = order == MV2H_ORDER_LINEAR ? 1 : 0;
    if (owner >= 0) {
        tp.owner_fixed = owner;
    } else {
        tp.owner_fixed = -1;
        tp.rs_blk = count / pof2;
    }
    LaunchCfg cfg{world().rl_grid, 2, st};
    tmark0(st);
    rc = launch_reduce_n(oi, dt->kind, srcs, nsrc, dst, count, dt->extent, tp, cfg);
    tmark1(st);
    if (rc) return rc;
    return finish(st, world().timing);
}

// ---------------------------------------------------------------------------
// part (2): device collectives
// ---------------------------------------------------------------------------
static int require_world() {
    World &w = world();
    if (!w.inited) {
        MV2_ERR("collective called before MPI_Init");
        return E_OTHER;
    }
    if (w.size > kMaxRanks) {
        MV2_ERR("device collectives support up to %d ranks per node (have %d)", kMaxRanks, w.size);
        return E_UNSUPPORTED;
    }
    return 0;
}

// staging: host or misaligned buffers go through device scratch (GPU does the work)
struct Staged {
    const char *send;
    char *recv;
    bool copy_back;
    void *user_recv;
    size_t bytes;
};

static int stage_in(const void *send, void *recv, size_t sbytes, size_t rbytes, bool in_place, hipStream_t st,
                    Staged &s) {
    s.copy_back = false;
    s.user_recv = recv;
    s.bytes = rbytes;
    const bool recv_ok = is_device(recv) && ((uintptr_t)recv % 16 == 0);
    if (recv_ok) {
        s.recv = (char *)recv;
    } else {
        s.recv = (char *)get_scratch(1, rbytes);
        if (!s.recv) return E_NO_MEM;
        s.copy_back = true;
        if (in_place) hipMemcpyAsync(s.recv, recv, rbytes, hipMemcpyDefault, st);
    }
    if (in_place) {
        s.send = s.recv;
    } else {
        const bool send_ok = is_device(send) && ((uintptr_t)send % 16 == 0);
        if (send_ok) {
            s.send = (const char *)send;
        } else {
            char *t = (char *)get_scratch(0, sbytes);
            if (!t) return E_NO_MEM;
            hipMemcpyAsync(t, send, sbytes, hipMemcpyDefault, st);
            s.send = t;
        }
    }
    return 0;
}

static void stage_out(const Staged &s, hipStream_t st) {
    if (s.copy_back) hipMemcpyAsync(s.user_recv, s.recv, s.bytes, hipMemcpyDefault, st);
}

static int allreduce_impl(const void *sendbuf, void *recvbuf, size_t count, const DtypeInfo *dt, int oi,
                          hipStream_t st) {
    World &w = world();
    const size_t bytes = count * (size_t)dt->extent;
    const bool in_place = sendbuf == (const void *)-1 || sendbuf == recvbuf;
    Staged s;
    int rc = stage_in(sendbuf, recvbuf, bytes, bytes, in_place, st, s);
    if (rc) return rc;
    const int n = w.size;
    if (n == 1 || oi == OP_NO_OP) {
        if (!in_place && oi != OP_NO_OP) hipMemcpyAsync(s.recv, s.send, bytes, hipMemcpyDeviceToDevice, st);
        stage_out(s, st);
        return finish(st, false);
    }
    if (oi == OP_REPLACE) {
        // result of REPLACE over ranks 0..n-1 in rank order: rank n-1's data; take the two-level
        // linear chain semantics: recv = x_{n-1} everywhere.  Realised as a broadcast from n-1.
        if (!in_place) hipMemcpyAsync(s.recv, s.send, bytes, hipMemcpyDeviceToDevice, st);
        stage_out(s, st);
        rc = finish(st, false);
        if (rc) return rc;
        return mv2h_bcast(recvbuf, bytes, n - 1, nullptr);
    }
    const TreeParams tp = make_tree(n, count, dt, w.rank);
    const uint64_t seq = ++w.seq;
    const uint64_t epoch = seq * 4 + 1;
    const size_t nvec = bytes / 16;
    const int gcap = grid_cap();
    if (bytes <= w.oneshot_max && bytes <= w.slot_bytes) {
        OneShotArgs a{};
        a.send = s.send;
        a.recv = s.recv;
        const size_t half = (size_t)kMaxRanks * w.slot_bytes;
        const size_t par = (seq & 1) * half;
        for (int j = 0; j < n; ++j) a.arena_peer.p[j] = w.peer_arena[j] + par;
        a.arena_own = w.arena + par;
        a.sig_peer = w.peer_sig;
        a.sig_own = w.sig;
        a.count = count;
        a.nvec = nvec;
        a.slot_bytes = w.slot_bytes;
        a.n = n;
        a.me = w.rank;
        a.tp = tp;
        a.epoch = epoch;
        a.err = w.h_err;
        a.timeout = w.timeout_ticks;
        int g = (int)((nvec + 511) / 512);
        g = std::max(1, std::min(g, std::min(gcap, 32)));
        LaunchCfg cfg = coll_cfg(g, st);
        tmark0(st);
        rc = launch_oneshot(oi, dt->kind, a, dt->extent, cfg);
        tmark1(st);
        if (rc) return rc;
        stage_out(s, st);
        return finish(st, w.timing);
    }
    // two-shot: exchange buffer descriptors (host), then one kernel
    if ((rc = publish(0, s.send))) return rc;
    if ((rc = publish(1, s.recv))) return rc;
    host_barrier();
    TwoShotArgs a{};
    for (int j = 0; j < n; ++j) {
        if (j == w.rank) {
            a.src.p[j] = s.send;
            a.agsrc.p[j] = s.recv;
            continue;
        }
        a.src.p[j] = peer_buffer(j, 0, &rc);
        if (rc) return rc;
        a.agsrc.p[j] = peer_buffer(j, 1, &rc);
        if (rc) return rc;
    }
    for (int j = n; j < kMaxRanks; ++j) {
        a.src.p[j] = a.src.p[0];
        a.agsrc.p[j] = a.agsrc.p[0];
    }
    a.recv = s.recv;
    a.sig_peer = w.peer_sig;
    a.sig_own = w.sig;
    a.count = count;
    a.nvec = nvec;
    a.n = n;
    a.me = w.rank;
    a.tp = tp;
    a.epoch = epoch;
    a.err = w.h_err;
    a.timeout = w.timeout_ticks;
    const size_t tv = (size_t)kThreads * twoshot_unroll(n);
    const size_t ntiles = (nvec + tv - 1) / tv;
    int g = (int)std::min<size_t>((ntiles + n - 1) / n, (size_t)gcap);
    if (g < 1) g = 1;
    LaunchCfg cfg = coll_cfg(g, st);
    tmark0(st);
    rc = launch_twoshot(oi, dt->kind, a, dt->extent, cfg);
    tmark1(st);
    if (rc) return rc;
    stage_out(s, st);
    return finish(st, w.timing);
}

int mv2h_allreduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream) {
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    if (count == 0) return 0;  // allreduce_osu.c:3730
    if ((rc = kind_supported(dt))) return rc;
    if ((rc = require_world())) return rc;
    return allreduce_impl(sendbuf, recvbuf, count, dt, op_index(op), pick_stream(stream));
}

int mv2h_reduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, int root, void *stream) {
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    if (count == 0) return 0;
    if ((rc = kind_supported(dt))) return rc;
    if ((rc = require_world())) return rc;
    World &w = world();
    if (root < 0 || root >= w.size) return E_ROOT;
    hipStream_t st = pick_stream(stream);
    const size_t bytes = count * (size_t)dt->extent;
    if (w.rank == root) return allreduce_impl(sendbuf, recvbuf, count, dt, op_index(op), st);
    // non-roots: recvbuf is insignificant; reduce into scratch
    void *tmp = get_scratch(2, bytes);
    if (!tmp) return E_NO_MEM;
    const void *src = sendbuf == (const void *)-1 ? recvbuf : sendbuf;
    return allreduce_impl(src, tmp, count, dt, op_index(op), st);
}

int mv2h_reduce_scatter(const void *sendbuf, void *recvbuf, const size_t *recvcounts, int dtype, int op,
                        void *stream) {
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    if ((rc = kind_supported(dt))) return rc;
    if ((rc = require_world())) return rc;
    World &w = world();
    const int n = w.size;
    size_t total = 0, off = 0;
    for (int j = 0; j < n; ++j) {
        if (j == w.rank) off = total;
        total += recvcounts[j];
    }
    if (total == 0) return 0;
    const int oi = op_index(op);
    hipStream_t st = pick_stream(stream);
    const size_t ext = dt->extent;
    const size_t mycnt = recvcounts[w.rank];
    const bool in_place = sendbuf == (const void *)-1;
    const void *send = in_place ? recvbuf : sendbuf;
    // sendbuf must be shareable device memory, 16-byte aligned: stage otherwise
    const char *s_dev = (const char *)send;
    if (!is_device(send) || (uintptr_t)send % 16) {
        char *t = (char *)get_scratch(0, total * ext);
        if (!t) return E_NO_MEM;
        hipMemcpyAsync(t, send, total * ext, hipMemcpyDefault, st);
        s_dev = t;
    }
    if (n == 1 || oi == OP_NO_OP || oi == OP_REPLACE) {
        if (!in_place && oi != OP_NO_OP) hipMemcpyAsync(recvbuf, s_dev, mycnt * ext, hipMemcpyDefault, st);
        return finish(st, false);
    }
    char *dst = (char *)get_scratch(1, total * ext);
    if (!dst) return E_NO_MEM;
    w.seq++;
    if ((rc = publish(0, s_dev))) return rc;
    host_barrier();
    RsArgs a{};
    for (int j = 0; j < n; ++j) {
        if (j == w.rank) {
            a.src.p[j] = s_dev;
            continue;
        }
        a.src.p[j] = peer_buffer(j, 0, &rc);
        if (rc) return rc;
    }
    for (int j = n; j < kMaxRanks; ++j) a.src.p[j] = a.src.p[0];
    a.dst = dst;
    a.sig_peer = w.peer_sig;
    a.sig_own = w.sig;
    a.off = off;
    a.cnt = mycnt;
    a.n = n;
    a.me = w.rank;
    TreeParams tp{};
    int pof2 = 1, lg = 0;
    while (pof2 * 2 <= n) { pof2 *= 2; ++lg; }
    tp.pof2 = pof2;
    tp.lg = lg;
    tp.rem = n - pof2;
    tp.linear = 1;
    a.tp = tp;
    a.epoch = w.seq * 4 + 1;
    a.err = w.h_err;
    a.timeout = w.timeout_ticks;
    const size_t nv = mycnt * ext / 16;
    int g = (int)std::min<size_t>((nv + 511) / 512, (size_t)grid_cap());
    if (g < 1) g = 1;
    LaunchCfg cfg = coll_cfg(g, st);
    tmark0(st);
    rc = launch_rs(oi, dt->kind, a, ext, cfg);
    tmark1(st);
    if (rc) return rc;
    if (mycnt) hipMemcpyAsync(recvbuf, dst + off * ext, mycnt * ext, hipMemcpyDefault, st);
    return finish(st, w.timing);
}

static int gather_impl(const char *const *srcs, char *dst, const size_t *dst_off, size_t bytes, hipStream_t st) {
    World &w = world();
    GatherArgs a{};
    for (int j = 0; j < kMaxRanks; ++j) a.src.p[j] = j < w.size ? srcs[j] : nullptr;
    for (int j = 0; j < kMaxRanks; ++j) a.dst_off[j] = j < w.size ? dst_off[j] : 0;
    a.dst = dst;
    a.bytes = bytes;
    a.sig_peer = w.peer_sig;
    a.sig_own = w.sig;
    a.n = w.size;
    a.me = w.rank;
    a.epoch = w.seq * 4 + 1;
    a.err = w.h_err;
    a.timeout = w.timeout_ticks;
    int g = (int)std::min<size_t>((bytes / 16 + 511) / 512, (size_t)grid_cap());
    if (g < 1) g = 1;
    LaunchCfg cfg = coll_cfg(g, st);
    tmark0(st);
    int rc = launch_gather(a, cfg);
    tmark1(st);
    if (rc) return rc;
    return finish(st, w.timing);
}

int mv2h_allgather(const void *sendbuf, void *recvbuf, size_t bytes, void *stream) {
    int rc;
    if ((rc = require_world())) return rc;
    if (bytes == 0) return 0;
    World &w = world();
    hipStream_t st = pick_stream(stream);
    const int n = w.size;
    const bool in_place = sendbuf == (const void *)-1;
    char *rdst = (char *)recvbuf;
    bool copy_back = false;
    if (!is_device(recvbuf)) {
        rdst = (char *)get_scratch(1, bytes * n);
        if (!rdst) return E_NO_MEM;
        copy_back = true;
        if (in_place) hipMemcpyAsync(rdst, recvbuf, bytes * n, hipMemcpyDefault, st);
    }
    const char *src = in_place ? rdst + (size_t)w.rank * bytes : (const char *)sendbuf;
    if (!in_place && !is_device(sendbuf)) {
        char *t = (char *)get_scratch(0, bytes);
        if (!t) return E_NO_MEM;
        hipMemcpyAsync(t, sendbuf, bytes, hipMemcpyDefault, st);
        src = t;
    }
    if (n == 1) {
        if (!in_place) hipMemcpyAsync(rdst, src, bytes, hipMemcpyDeviceToDevice, st);
    } else {
        w.seq++;
        if ((rc = publish(0, src))) return rc;
        host_barrier();
        const char *srcs[kMaxRanks];
        size_t offs[kMaxRanks];
        for (int j = 0; j < n; ++j) {
            offs[j] = (size_t)j * bytes;
            if (j == w.rank) {
                srcs[j] = in_place ? nullptr : src;
                continue;
            }
            srcs[j] = peer_buffer(j, 0, &rc);
            if (rc) return rc;
        }
        if ((rc = gather_impl(srcs, rdst, offs, bytes, st))) return rc;
    }
    if (copy_back) hipMemcpyAsync(recvbuf, rdst, bytes * n, hipMemcpyDefault, st);
    return finish(st, false);
}

int mv2h_bcast(void *buffer, size_t bytes, int root, void *stream) {
    int rc;
    if ((rc = require_world())) return rc;
    if (bytes == 0) return 0;
    World &w = world();
    if (root < 0 || root >= w.size) return E_ROOT;
    if (w.size == 1) return 0;
    hipStream_t st = pick_stream(stream);
    char *buf = (char *)buffer;
    bool copy_back = false;
    if (!is_device(buffer)) {
        buf = (char *)get_scratch(1, bytes);
        if (!buf) return E_NO_MEM;
        copy_back = w.rank != root;
        if (w.rank == root) hipMemcpyAsync(buf, buffer, bytes, hipMemcpyHostToDevice, st);
    }
    w.seq++;
    if (w.rank == root && (rc = publish(0, buf))) return rc;
    host_barrier();
    const char *srcs[kMaxRanks] = {};
    size_t offs[kMaxRanks] = {};
    if (w.rank != root) {
        srcs[root] = peer_buffer(root, 0, &rc);
        if (rc) return rc;
    }
    if ((rc = gather_impl(srcs, buf, offs, bytes, st))) return rc;
    if (copy_back) {
        hipMemcpyAsync(buffer, buf, bytes, hipMemcpyDeviceToHost, st);
        return finish(st, false);
    }
    return 0;
}

// ---------------------------------------------------------------------------
// part (3): strided pack / unpack
// ---------------------------------------------------------------------------
int mv2h_pack_strided(const void *src, void *dst, size_t nblocks, size_t blk, size_t stride, void *stream) {
    int rc;
    if ((rc = ensure_init_for_device())) return rc;
    hipStream_t st = pick_stream(stream);
    tmark0(st);
    rc = launch_pack_strided(src, dst, nblocks, blk, stride, 0, st);
    tmark1(st);
    if (rc) return rc;
    return finish(st, world().timing);
}

int mv2h_unpack_strided(const void *src, void *dst, size_t nblocks, size_t blk, size_t stride, void *stream) {
    int rc;
    if ((rc = ensure_init_for_device())) return rc;
    hipStream_t st = pick_stream(stream);
    tmark0(st);
    rc = launch_pack_strided(src, dst, nblocks, blk, stride, 1, st);
    tmark1(st);
    if (rc) return rc;
    return finish(st, world().timing);
}

}  // extern "C"
