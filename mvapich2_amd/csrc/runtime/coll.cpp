// coll.cpp — the mv2h_* C-ABI (include/mv2h.h): op layer entry points and
// host orchestration of the device collectives.
//
// Every reducing call first takes the reference's one-node algorithm choice
// (orders.cpp plan_allreduce / plan_reduce / plan_reduce_scatter, restating
// MPIR_Allreduce_index_tuned_intra_MV2 allreduce_osu.c:3015-3420,
// MPIR_Reduce_index_tuned_intra_MV2 reduce_osu.c:2391-2660 and
// MPIR_Reduce_scatter_MV2 red_scat_osu.c:1859-1896) and then runs that
// algorithm's operand order on the device (specialised LINEAR / ring /
// butterfly evaluators, or per-element programs).  The data path is
// MI355X-native: one-shot push through uncached IPC arenas for small messages,
// pipelined direct reduce-scatter + all-gather pushed into peers' arenas over
// xGMI for large ones (coll/pipe.h), tiled by the MPI_Init autotune.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <chrono>
#include <vector>
#include <unistd.h>

#include "../../../include/mv2h.h"
#include "log.h"
#include "orders.h"
#include "pvars.h"
#include "world.h"
#include "internode.h"

namespace mv2 {

int log_rank() { return world().grank; }  // the job's rank (a node's local rank 0 is not unique)
bool log_debug_on() {
    static int on = -1;
    if (on < 0) {
        const char *v = getenv("MV2AMD_DEBUG");
        on = (v && *v && *v != '0') ? 1 : 0;
    }
    return on == 1;
}

// The stream of a call.  Every collective kernel of this process shares the arenas, flag
// epochs and slot parities, which the host hands out in call order, so the kernels must also
// run in call order whatever stream each call names.  One event carries the order: a call on
// a caller's stream records it on that stream when it ends (stream_tail — the caller may
// destroy the stream afterwards, so the library never touches it again), a call on the
// library's own stream records it lazily when the next call names another stream; a call on
// a stream other than the previous one first waits for it.  Calls that stay on one stream
// pay nothing for the order.  (A caller's stream handle reused after hipStreamDestroy is
// safe: the destroy drains the stream's queue first.)
static hipStream_t pick_stream(void *s) {
    World &w = world();
    hipStream_t st = s ? (hipStream_t)s : w.stream;
    if (st == w.stream) w.stream_hip_busy = true;  // runtime/aql.cpp consults HIP before its next dispatch
    if (w.graph) return st;  // graph lane: disjoint arenas and epochs, ordered by the graph itself
    if (w.last_st && st != w.last_st) {
        if (!w.sw_ev) hipEventCreateWithFlags(&w.sw_ev, hipEventDisableTiming);
        if (w.sw_ev) {
            if (w.last_st == w.stream && st != w.stream) hipEventRecord(w.sw_ev, w.stream);
            hipStreamWaitEvent(st, w.sw_ev, 0);
        }
    }
    w.last_st = st;
    return st;
}
static void stream_tail(hipStream_t st) {
    World &w = world();
    if (st == w.stream || w.graph) return;
    if (!w.sw_ev) hipEventCreateWithFlags(&w.sw_ev, hipEventDisableTiming);
    if (w.sw_ev) hipEventRecord(w.sw_ev, st);
}

// Host-side profile of blocking calls (MV2AMD_HOST_PROFILE=1, printed at
// MPI_Finalize): time from API entry to the kernel launch (argument checks,
// plan, staging), inside hipLaunchKernel, and from the launch to the
// completion word (kernel run + peers' arrival).
struct HostProf {
    int on = -1;
    uint64_t calls = 0, pre_ns = 0, launch_ns = 0, wait_ns = 0;
    uint64_t t_entry = 0, t_l0 = 0, t_l1 = 0;
};
static HostProf g_hp;
static inline uint64_t now_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}
static inline bool hp_on() {
    if (g_hp.on < 0) {
        const char *v = getenv("MV2AMD_HOST_PROFILE");
        g_hp.on = v && atoi(v) > 0 ? atoi(v) : 0;
    }
    return g_hp.on;
}
static bool g_call_start = true;  // tmark0: record ev0 at the first launch of this API call
static inline void hp_entry() {
    g_call_start = true;
    beacon(BC_ENTRY, true);
    if (hp_on()) g_hp.t_entry = now_ns();
}
static inline void hp_done() {
    if (!hp_on() || !g_hp.t_entry || !g_hp.t_l1) return;
    const uint64_t t = now_ns();
    // MV2AMD_HOST_PROFILE=k > 1: the first k - 1 calls (warm-up, first-launch code loading) are
    // left out of the means
    static uint64_t seen = 0;
    if (++seen < (uint64_t)g_hp.on) {
        g_hp.t_entry = g_hp.t_l0 = g_hp.t_l1 = 0;
        return;
    }
    ++g_hp.calls;
    g_hp.pre_ns += g_hp.t_l0 - g_hp.t_entry;
    g_hp.launch_ns += g_hp.t_l1 - g_hp.t_l0;
    g_hp.wait_ns += t - g_hp.t_l1;
    g_hp.t_entry = g_hp.t_l0 = g_hp.t_l1 = 0;
}
void host_prof_report() {
    if (!hp_on() || !g_hp.calls) return;
    const double c = (double)g_hp.calls * 1e3;
    fprintf(stderr, "[mv2amd rank %d] host profile: %llu calls, entry->launch %.3f us, launch %.3f us, launch->done %.3f us\n",
            world().rank, (unsigned long long)g_hp.calls, g_hp.pre_ns / c, g_hp.launch_ns / c, g_hp.wait_ns / c);
}


// Completion word for the kernel about to be launched on `st` as the call's
// last stream operation (only the library's own stream; cleared again by
// any copy enqueued after it, see enq_copy).
// Test hooks (mv2h_set_tuning): "withhold_done" = k makes the next k armed kernels run without
// their word (the host still waits for it: the missed-word path of wait_done), "fake_split" = k
// marks the next k words as raised by a kernel whose block groups ran on several XCDs.
static int g_withhold_done = 0, g_fake_split = 0;

static Done arm_done(hipStream_t st) {
    World &w = world();
    if (w.sync_mode != 0 || !w.done_flag || st != w.stream || w.enqueue) return Done{nullptr, nullptr, 0};
    w.pending = ++w.done_seq;
    if (g_fake_split > 0) {
        --g_fake_split;
        __atomic_store_n(w.done_flag + 1, w.pending, __ATOMIC_RELEASE);
    }
    if (g_withhold_done > 0) {
        --g_withhold_done;
        return Done{nullptr, nullptr, 0};
    }
    return Done{w.done_ctr, w.done_flag, w.pending};
}

static inline hipError_t enq_copy(void *dst, const void *src, size_t bytes, hipStream_t st) {
    beacon(BC_COPY_OUT);
    world().pending = 0;
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st);
}

// A completion word whose kernel ran a block group over more than one XCD (device_util.h
// block_done wrote its seq into done_flag[1] too): that group's L2 write-back did not cover every
// block, so the call completes with a stream synchronisation (the kernel's end releases every
// XCD's L2) before the host returns.  Counted (done_xcd_split) and reported once per process.
static hipError_t settle_split(hipStream_t st) {
    World &w = world();
    const uint64_t s = __atomic_load_n(w.done_flag + 1, __ATOMIC_ACQUIRE);
    if (s <= w.split_seen) return hipSuccess;
    w.split_seen = s;
    if (w.done_xcd_split++ == 0)
        fprintf(stderr, "[mv2amd rank %d] warning: a kernel's workgroups of one group ran on several XCDs; "
                        "completing such calls with a stream synchronisation (counted in done_xcd_split)\n",
                log_rank());
    return hipStreamSynchronize(st);
}

// Wait for the armed completion word; fall back to the stream when the
// kernel ended without raising it (should not happen: counters are reset).
// The word is the normal path: the stream is consulted only once the word is
// 200 us late, then every 100 us (a hipStreamQuery costs ~3 us of host time,
// and one in flight when the word lands delays the return by that much).
// Every fallback is counted and the first missed word of the process is reported (a missed word
// would otherwise be invisible in every record): done_queried -- the stream was consulted at least
// once (any call whose kernel runs longer than 200 us, e.g. a 256 MiB allreduce on a shared GPU);
// done_late -- the stream already reported the kernel finished when the word was seen (the word
// trailed the kernel's end); done_missed -- the kernel had ended without raising the word.
static hipError_t wait_done(hipStream_t st, uint64_t want) {
    World &w = world();
    uint64_t next_query = 0;
    bool queried = false;
    for (unsigned spins = 0;; ++spins) {
        if (__atomic_load_n(w.done_flag, __ATOMIC_ACQUIRE) >= want) return settle_split(st);
        if ((spins & 255u) == 0) {
            const uint64_t t = now_ns();
            if (!next_query) next_query = t + 200000;
            if (t < next_query) continue;
            next_query = t + 100000;
            if (!queried) {
                queried = true;
                ++w.done_queried;
            }
            const hipError_t q = hipStreamQuery(st);
            if (q == hipErrorNotReady) continue;
            if (__atomic_load_n(w.done_flag, __ATOMIC_ACQUIRE) >= want) {
                if (q == hipSuccess) ++w.done_late;
                return settle_split(st);
            }
            if (q == hipSuccess) {
                if (w.done_missed++ == 0)
                    fprintf(stderr, "[mv2amd rank %d] warning: a kernel finished without raising its completion word "
                                    "(call %llu); completing by stream synchronisation, counters reset (counted in done_missed)\n",
                            log_rank(), (unsigned long long)want);
                hipMemsetAsync(w.done_ctr, 0, kDoneBytes, st);
                return hipStreamSynchronize(st);
            }
            return q;
        }
    }
}

static void log_epochs(uint64_t lo, uint64_t hi, hipStream_t st) {
    World &w = world();
    w.epoch_log[w.epoch_pos++ % 8] = World::EpochRec{w.api_calls, lo, hi, st != w.stream};
}

// The waited slot of every rank in `mask` as it is in memory now (read by a copy on a stream of
// its own, after the kernel gave up): a value above the one the kernel last saw means its loads
// were served stale; the same value means the peer's flag store never landed.
static void report_slot_now(int blk, unsigned mask) {
    World &w = world();
    if (!w.sig || blk < 0 || blk >= kMaxBlocks) return;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    uint64_t *h = nullptr;
    if (hipHostMalloc((void **)&h, kMaxRanks * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        hipStreamDestroy(s);
        return;
    }
    bool ok = true;
    for (int j = 0; j < kMaxRanks && ok; ++j)
        if ((mask >> j) & 1u)
            ok = hipMemcpyAsync(h + j, w.sig + (size_t)j * kMaxBlocks + blk, sizeof(uint64_t), hipMemcpyDeviceToHost, s) ==
                 hipSuccess;
    const uint64_t t0 = now_ns();
    hipError_t q = hipErrorNotReady;
    while (ok && (q = hipStreamQuery(s)) == hipErrorNotReady && now_ns() - t0 < 2000000000ull) usleep(100);
    if (ok && q == hipSuccess) {
        char line[256];
        int o = 0;
        for (int j = 0; j < kMaxRanks && o < (int)sizeof(line) - 40; ++j)
            if ((mask >> j) & 1u) o += snprintf(line + o, sizeof(line) - o, " r%d=%llu", j, (unsigned long long)h[j]);
        line[o] = 0;
        MV2_ERR("  the waited slot now (host copy):%s", line);
    }
    (void)hipGetLastError();
    if (q != hipErrorNotReady) {  // a copy still in flight keeps its buffers
        hipHostFree(h);
        hipStreamDestroy(s);
    }
}

// A kernel gave up waiting for a peer (device_util.h wait_mask): report what it waited for —
// the epoch, the ranks and the flag values it last saw from each, next to this rank's host
// counters — so a failure tells a late peer (flag = an earlier epoch of the same call
// sequence) from a peer whose call sequence diverged (flags of another call's epochs).
static int check_err_word() {
    World &w = world();
    if (!w.h_err || !__atomic_load_n(w.h_err, __ATOMIC_ACQUIRE)) return 0;
    int *e = w.h_err;
    const uint64_t ep = (uint64_t)(uint32_t)e[2] | ((uint64_t)(uint32_t)e[3] << 32);
    char seen[256];
    int o = 0;
    for (int j = 0; j < kMaxRanks && o < (int)sizeof(seen) - 40; ++j)
        if (((unsigned)e[4] >> j) & 1u) {
            const uint64_t v = (uint64_t)(uint32_t)e[8 + 2 * j] | ((uint64_t)(uint32_t)e[9 + 2 * j] << 32);
            o += snprintf(seen + o, sizeof(seen) - o, " r%d=%llu", j, (unsigned long long)v);
        }
    seen[o] = 0;
    MV2_ERR("device collective timed out waiting for a peer (MV2AMD_TIMEOUT_S): workgroup %d waited for epoch "
            "%llu from ranks 0x%x; flags seen:%s; host epoch %llu, round %llu, one-shot calls %llu, call %llu",
            e[1], (unsigned long long)ep, (unsigned)e[4], seen, (unsigned long long)w.epoch, (unsigned long long)w.round,
            (unsigned long long)w.os_calls, (unsigned long long)w.done_seq);
    {
        char line[512];
        int o = 0;
        for (unsigned k = w.epoch_pos > 8 ? w.epoch_pos - 8 : 0; k < w.epoch_pos && o < (int)sizeof(line) - 80; ++k) {
            const World::EpochRec &r = w.epoch_log[k % 8];
            o += snprintf(line + o, sizeof(line) - o, " %llu:%llu-%llu%s%s", (unsigned long long)r.call,
                          (unsigned long long)r.lo, (unsigned long long)r.hi, r.user_stream ? "(caller's stream)" : "",
                          r.lo <= ep && ep <= r.hi ? "<-" : "");
        }
        line[o] = 0;
        MV2_ERR("  this rank's last launches with flag epochs (call:epochs, <- the waiting one):%s", line);
    }
    report_slot_now(e[1], (unsigned)e[4]);
    // where each late peer's host is now (its beacon in the control segment), next to this rank's
    if (w.shm) {
        const uint64_t t = now_ns();
        for (int j = 0; j < w.size && j < kMaxRanks; ++j) {
            const uint64_t v = (uint64_t)(uint32_t)e[8 + 2 * j] | ((uint64_t)(uint32_t)e[9 + 2 * j] << 32);
            if (j != w.rank && !((((unsigned)e[4] >> j) & 1u) && v < ep)) continue;
            const uint64_t b = w.shm->r[j].beacon.load(std::memory_order_relaxed);
            const uint64_t bt = w.shm->r[j].beacon_ns.load(std::memory_order_relaxed);
            MV2_ERR("  %s local rank %d: library call %llu, %s, for %.1f ms", j == w.rank ? "this is" : "late peer:", j,
                    (unsigned long long)(b >> 8), beacon_name((int)(b & 0xff)), bt && t > bt ? (t - bt) / 1e6 : 0.0);
            beacon_report(j, t);
        }
    }
    memset(e + 1, 0, (kErrWords - 1) * sizeof(int));
    __atomic_store_n(e, 0, __ATOMIC_RELEASE);
    return E_OTHER;
}

static int finish(hipStream_t st, bool timed) {
    World &w = world();
    hipError_t e;
    const uint64_t want = w.pending;
    w.pending = 0;
    stream_tail(st);
    if (w.enqueue) return 0;  // stream-ordered: the caller's stream carries the completion
    if (w.defer && want) {  // nonblocking initiation: the ticket waits later
        w.deferred = want;
        return 0;
    }
    if (w.defer) w.deferred = 0;
    beacon(BC_WAIT);
    if (want) {
        e = wait_done(st, want);
        if (e == hipSuccess && timed) e = hipEventSynchronize(w.ev1);
    } else {
        e = hipStreamSynchronize(st);
    }
    if (e != hipSuccess) {
        MV2_ERR("hipStreamSynchronize failed: %s", hipGetErrorString(hipGetLastError()));
        return E_INTERN;
    }
    if (timed) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, w.ev0, w.ev1);
        w.last_ms = ms;
    }
    if (check_err_word()) return E_OTHER;
    beacon(BC_DONE);
    hp_done();
    return 0;
}

// kernel-time events bracket the call's first launch to its last (calls made of several
// launches: ring main part + remainder, staged copies)
static inline void tmark0(hipStream_t st) {
    if (g_call_start) beacon(BC_LAUNCH);
    if (world().timing && g_call_start) hipEventRecord(world().ev0, st);
    g_call_start = false;
    if (hp_on() && g_hp.t_entry && !g_hp.t_l0) g_hp.t_l0 = now_ns();
}
static inline void tmark1(hipStream_t st) {
    beacon(BC_LAUNCHED);
    if (world().timing) hipEventRecord(world().ev1, st);
    if (hp_on() && g_hp.t_entry) g_hp.t_l1 = now_ns();
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

// The call's last copy, device to device, as a copy kernel that raises the completion word:
// a hipMemcpyAsync cannot raise it, and without it finish() falls back to a stream
// synchronisation (several us at small sizes).  Other copies keep enq_copy.
static hipError_t enq_copy_last(void *dst, const void *src, size_t bytes, hipStream_t st) {
    constexpr size_t kKernelCopyMax = (size_t)4 << 20;
    if (bytes && bytes <= kKernelCopyMax && is_device(dst) && is_device(src)) {
        const Done d = arm_done(st);
        if (d.flag) {
            beacon(BC_COPY_OUT);
            if (launch_pack_strided(src, dst, 1, bytes, bytes, 0, st, d) == 0) return hipSuccess;
            world().pending = 0;  // no kernel will raise the word: finish() must not wait for it
            MV2_ERR("launching the result copy-out failed: %s", hipGetErrorString(hipGetLastError()));
            return hipErrorLaunchFailure;
        }
    }
    return enq_copy(dst, src, bytes, st);
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
// reduction order (algorithm choice and programs: orders.cpp)
// ---------------------------------------------------------------------------
static TreeParams tree_base(int n) {
    TreeParams tp{};
    int pof2 = 1, lg = 0;
    while (pof2 * 2 <= n) { pof2 *= 2; ++lg; }
    tp.pof2 = pof2;
    tp.lg = lg;
    tp.rem = n - pof2;
    return tp;
}

// pt2pt_rs order on the specialised butterfly evaluator: recursive halving
// with owner bitrev(block), or recursive doubling (count < pof2, or the
// pt2pt_rd algorithm) where each rank keeps its own result and even ranks
// below 2*rem take their odd partner's (allreduce_osu.c:585-600, :1003-1030)
static TreeParams tree_rs(int n, size_t count, int me, bool force_rd) {
    TreeParams tp = tree_base(n);
    tp.linear = 0;
    if (!force_rd && count >= (size_t)tp.pof2) {
        tp.owner_fixed = -1;
        tp.rs_blk = count / tp.pof2;
    } else {
        int r = me;
        if (r < 2 * tp.rem && r % 2 == 0) r = r + 1;
        tp.owner_fixed = (r < 2 * tp.rem) ? r / 2 : r - tp.rem;
    }
    return tp;
}

// A program set whose every program is acc = ((x0 . x1) . x2) ... (the degree-4 tree over one
// group of <= 4 ranks, and any other algorithm that reduces to it) runs on the specialised
// LINEAR evaluator instead of the program kernel: same operands in the same order.
static bool progs_are_linear(const ProgSet &ps, int n) {
    if (ps.nprog < 1) return false;
    for (int k = 0; k < ps.nprog; ++k) {
        const Prog &q = ps.p[k];
        if (q.nsteps != n - 1 || q.res != 0) return false;
        for (int s = 0; s < n - 1; ++s)
            if (q.dst[s] != 0 || q.src[s] != s + 1) return false;
    }
    return true;
}

// The two-level degree-d tree (d < n) as a program: each group leader g reduces g+1 .. g+d-1,
// then rank 0 reduces the leaders d, 2d, ... in order.  Returns d when `ps` is that program.
static int progs_grouped(const ProgSet &ps, int n) {
    if (ps.nprog != 1) return 0;
    const Prog &q = ps.p[0];
    for (int d = 2; d < n; ++d) {
        uint8_t dst[kMaxRanks], src[kMaxRanks];
        int k = 0;
        for (int g = 0; g < n; g += d)
            for (int m = g + 1; m < g + d && m < n; ++m) dst[k] = (uint8_t)g, src[k++] = (uint8_t)m;
        for (int g = d; g < n; g += d) dst[k] = 0, src[k++] = (uint8_t)g;
        if (k != q.nsteps || q.res != 0) continue;
        bool same = true;
        for (int s = 0; s < k && same; ++s) same = q.dst[s] == dst[s] && q.src[s] == src[s];
        if (same) return d;
    }
    return 0;
}

static TreeParams tree_from_plan(const Plan &p, int n, size_t count, int me) {
    if (p.algo != ALG_PT2PT_RS && p.algo != ALG_PT2PT_RD && p.algo != ALG_SHMEM_LINEAR && progs_are_linear(p.ps, n)) {
        TreeParams tp = tree_base(n);
        tp.linear = 1;
        return tp;
    }
    switch (p.algo) {
    case ALG_PT2PT_RS: return tree_rs(n, count, me, false);
    case ALG_PT2PT_RD: return tree_rs(n, count, me, true);
    case ALG_SHMEM_LINEAR:
        if (!p.inner) {
            TreeParams tp = tree_base(n);
            tp.linear = 1;
            return tp;
        }
        [[fallthrough]];  // reduce_shmem from the shmem slot on: the inner reduce's programs
    default: {
        TreeParams tp = tree_base(n);
        tp.linear = 4;
        tp.ps = p.ps;
        return tp;
    }
    }
}

static void log_plan(const char *coll, const Plan &p, size_t count) {
    MV2_DEBUG("%s count %zu -> %s%s%s", coll, count, algo_name(p.algo), p.inner ? " / " : "",
              p.inner ? algo_name(p.inner) : "");
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
// pipelined collectives (coll/pipe.h)
// ---------------------------------------------------------------------------
struct PipeGeom {
    int grid;
    size_t tsub, tseg;
    int nrounds;
};

// Grid and per-block range of a pipelined call.  A pure function of the
// message geometry and of values every rank shares (CU count, ranks per GPU,
// tuning knobs), so block b of every rank handles the same bytes.
static long env_long_coll(const char *name, long dflt);
static PipeGeom pipe_geom(size_t maxlen) {
    World &w = world();
    int cap = std::min(kPipeMaxGrid, xcd_fair_cap(1, w.cus, w.nshare));  // k_pipe: one block per CU
    cap = std::min(cap, std::max(1, w.pipe_grid));
    // the smallest per-workgroup tile: 4 KiB (measured against 8 and 16 KiB: a small message
    // spread over more workgroups leaves each thread fewer dependent memory round trips per
    // phase; 1 MiB at 4 shared ranks 37.1 -> 28.7 us).  MV2AMD_PIPE_MIN_SUB overrides it.
    static const size_t kMinSub = (size_t)std::max(4096L, env_long_coll("MV2AMD_PIPE_MIN_SUB", 4096)) & ~(size_t)4095;
    PipeGeom g{};
    g.grid = (int)std::min<size_t>((size_t)cap, std::max<size_t>(1, (maxlen + kMinSub - 1) / kMinSub));
    size_t tsub = (maxlen + g.grid - 1) / g.grid;
    tsub = (tsub + 4095) & ~(size_t)4095;
    // a round's slot (grid x tsub) must fit the kPipeSlot bytes of an arena slot
    const size_t sub_cap = std::min(kPipeSlot / (size_t)g.grid, std::max<size_t>(4096, w.pipe_sub));
    g.tsub = std::min(tsub, sub_cap & ~(size_t)4095);
    g.tseg = (size_t)g.grid * g.tsub;
    g.nrounds = (int)((maxlen + g.tseg - 1) / g.tseg);
    return g;
}

// the tiling a segment of seg_bytes runs with (MPI_Init's report)
void pipe_tiling_for(size_t seg_bytes, int *grid, size_t *tsub) {
    const PipeGeom g = pipe_geom(seg_bytes);
    *grid = g.grid;
    *tsub = g.tsub;
}

// n contiguous 16-byte-aligned segments of a `bytes` buffer (the last may be short or empty)
static void even_segments(PipeArgs &a, size_t bytes, int n) {
    const size_t seg = (((bytes + n - 1) / n) + 15) & ~(size_t)15;
    for (int j = 0; j < n; ++j) {
        const size_t off = std::min((size_t)j * seg, bytes);
        a.seg_off[j] = a.recv_off[j] = off;
        a.seg_len[j] = std::min(seg, bytes - off);
    }
}

// Fill the runtime part of `a`, reserve rounds/epochs and launch (no sync).
// dt == nullptr: data-movement modes (AG / BC).
static int run_pipe(PipeArgs &a, int oi, const DtypeInfo *dt, hipStream_t st) {
    World &w = world();
    a.n = w.size;
    a.me = w.rank;
    size_t maxlen = 0;
    for (int j = 0; j < a.n; ++j) maxlen = std::max(maxlen, a.seg_len[j]);
    if (maxlen == 0) return 0;  // every rank sees the same geometry
    const PipeGeom g = pipe_geom(maxlen);
    a.tsub = g.tsub;
    a.tseg = g.tseg;
    a.nrounds = g.nrounds;
    a.rnt = w.pipe_rnt;
    if (w.graph) {  // graph lane: own arenas and flags; epochs and parities from the device
        a.rs_peer = w.g_peer_rs;
        a.ag_peer = w.g_peer_ag;
        a.sig_peer = w.g_peer_sig;
        a.sig_own = w.g_sig;
        a.dseq = w.dseq;
    } else {
        a.rs_peer = w.peer_rs;
        a.ag_peer = w.peer_ag;
        a.sig_peer = w.peer_sig;
        a.sig_own = w.sig;
        a.round0 = w.round;
        w.round += (uint64_t)g.nrounds;
        a.epoch0 = w.epoch + 1;
        w.epoch += 2 * (uint64_t)g.nrounds;
        log_epochs(a.epoch0, w.epoch, st);
    }
    a.err = w.h_err;
    a.timeout = w.timeout_ticks;
    a.light = w.light_release;
    a.done = arm_done(st);
    MV2_DEBUG("pipe mode %d grid %d tsub %zu rounds %d maxlen %zu", a.mode, g.grid, g.tsub, g.nrounds, maxlen);
    LaunchCfg cfg = coll_cfg(g.grid, st);
    tmark0(st);
    const int rc = dt ? launch_pipe_reduce(oi, dt->kind, a, cfg) : launch_pipe_copy(a, cfg);
    tmark1(st);
    return rc;
}

// The one-shot kernels' per-call part: this call's arena half and flag epoch (or, on the graph
// lane, where the kernel reads them), the peers, the error word, the completion word.
static void oneshot_common(OneShotArgs &a, hipStream_t st) {
    World &w = world();
    const int n = w.size;
    const size_t half = (size_t)kMaxRanks * w.slot_bytes;
    if (w.graph) {  // graph lane: the kernel picks the half and the epoch from the device
        for (int j = 0; j < n; ++j) a.arena_peer.p[j] = w.g_peer_arena[j];
        a.arena_own = w.g_arena;
        a.sig_peer = w.g_peer_sig;
        a.sig_own = w.g_sig;
        a.dseq = w.dseq;
        a.half = half;
    } else {
        const size_t par = (w.os_calls++ & 1) * half;
        for (int j = 0; j < n; ++j) a.arena_peer.p[j] = w.peer_arena[j] + par;
        a.arena_own = w.arena + par;
        a.sig_peer = w.peer_sig;
        a.sig_own = w.sig;
        a.epoch = ++w.epoch;
        log_epochs(a.epoch, a.epoch, st);
    }
    a.slot_bytes = w.slot_bytes;
    a.n = n;
    a.me = w.rank;
    a.err = w.h_err;
    a.timeout = w.timeout_ticks;
    a.light = w.light_release;
    a.done = arm_done(st);
}

static long env_long_coll(const char *name, long dflt);
// one 16-B vector per thread of a 256-thread workgroup, up to 64 workgroups (256 KiB): the
// one-shot kernels are latency-bound, and each further vector a thread owns costs it another
// dependent memory round trip (MV2AMD_ONESHOT_VECS_PER_WG / _MAX_WG override)
static int oneshot_grid(size_t nvec, int gcap) {
    static const long vpw = std::max(64L, env_long_coll("MV2AMD_ONESHOT_VECS_PER_WG", 256));
    static const int wmax = (int)std::min(1024L, std::max(1L, env_long_coll("MV2AMD_ONESHOT_MAX_WG", 64)));
    const int g = (int)((nvec + vpw - 1) / vpw);
    return std::max(1, std::min(g, std::min(gcap, wmax)));
}

}  // namespace mv2

// the node-level allreduce (defined with the C-ABI below): MPI_Init's self-test and tiling
// probe run on this node's world, before any inter-node link exists
extern "C" {
static int allreduce_entry(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream);
}

namespace mv2 {

// Init-time choice of the pipelined kernels' tiling (workgroups x bytes per workgroup per
// round) on this node's links.  The link rate of a peer store stream and the cost of a
// round's flag exchange are properties of the machine, not of the message, so MPI_Init times
// the headline operation — a 256 MiB fp32 SUM MPI_Allreduce, which takes the ring-wrapper
// order — under a few tilings on every rank, takes each candidate's maximum over ranks through
// the host control segment, and every rank adopts the same minimum (kernels pair workgroup b
// of every rank, so the grid must agree).  The tiling never changes a result: the reduction
// order is fixed per element by the plan.  Runs with one rank per GPU (xGMI) unless
// MV2AMD_PIPE_AUTOTUNE=0, or on a shared GPU with MV2AMD_PIPE_AUTOTUNE=1; an explicit
// MV2AMD_PIPE_GRID / MV2AMD_PIPE_SUB disables it.
int oneshot_autotune();

static long env_long_coll(const char *name, long dflt) {
    const char *v = getenv(name);
    return v && *v ? atol(v) : dflt;
}

int pipe_autotune() {
    World &w = world();
    const char *ev = getenv("MV2AMD_PIPE_AUTOTUNE");
    const long mode = ev && *ev ? atol(ev) : -1;
    if (mode == 0 || (mode < 0 && w.nshare > 1) || w.size < 2 || getenv("MV2AMD_PIPE_GRID") ||
        getenv("MV2AMD_PIPE_SUB"))
        return 0;
    const char *eb = getenv("MV2AMD_PIPE_AUTOTUNE_BYTES");
    const size_t count = (size_t)(eb && atol(eb) > 0 ? atol(eb) : 256L << 20) / 4;
    const int MPI_FLOAT_H = 0x4c00040a, MPI_SUM_H = 0x58000003;
    void *sb = nullptr, *rb = nullptr;
    if (hipMalloc(&sb, count * 4) != hipSuccess || hipMalloc(&rb, count * 4) != hipSuccess) {
        if (sb) hipFree(sb);
        MV2_DEBUG("pipe autotune skipped: no device memory for the probe buffers");
        return 0;
    }
    hipMemset(sb, 0, count * 4);
    hipDeviceSynchronize();
    // tilings x the flavour of the stores into peers' arenas (non-temporal or plain: how the
    // fabric combines them is a property of the links, measured rather than assumed)
    // (256 x 16 KiB: 8 rounds of a 32 MiB segment at 8 ranks, the deepest pipeline)
    static const int kGrid[] = {256, 256, 256, 256, 128, 128, 64};
    static const size_t kSub[] = {128 << 10, 64 << 10, 32 << 10, 16 << 10, 256 << 10, 128 << 10, 512 << 10};
    constexpr int kTilings = (int)(sizeof(kGrid) / sizeof(kGrid[0]));
    const int g0 = w.pipe_grid, r0 = w.pipe_rnt;
    const size_t s0 = w.pipe_sub;
    int nc = 0;
    int rc = 0;
    // time budget (MV2AMD_PIPE_AUTOTUNE_BUDGET_MS, default 3 s of MPI_Init): rank 0 ends the
    // probe when it is spent and every rank stops at the same candidate (one barrier publishes
    // the decision, a second one keeps rank 0 from rewriting it before every rank has read it)
    const double budget_ms = (double)env_long_coll("MV2AMD_PIPE_AUTOTUNE_BUDGET_MS", 3000);
    const auto t_begin = std::chrono::steady_clock::now();
    for (int c = 0; c < 2 * kTilings && nc < kTuneMax; ++c) {
        if (w.rank == 0)
            w.shm->tune_stop.store(
                nc > 0 && std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_begin).count() >
                              budget_ms ? 1 : 0);
        host_barrier();
        const bool stop = w.shm->tune_stop.load() != 0;
        host_barrier();
        if (stop) break;
        w.pipe_grid = kGrid[c % kTilings];
        w.pipe_sub = kSub[c % kTilings];
        w.pipe_rnt = c < kTilings ? 1 : 0;
        const PipeGeom g = pipe_geom((count * 4 + w.size - 1) / w.size);
        bool dup = false;  // the grid cap of a shared GPU can fold candidates together
        for (int k = 0; k < nc; ++k)
            dup |= w.tune_grid[k] == g.grid && w.tune_sub[k] == g.tsub && w.tune_rnt[k] == w.pipe_rnt;
        if (dup) continue;
        w.tune_grid[nc] = g.grid;
        w.tune_sub[nc] = g.tsub;
        w.tune_rnt[nc] = w.pipe_rnt;
        double best = 1e30;
        for (int it = 0; it < 4 && !rc; ++it) {  // the first call warms the tiling up
            host_barrier();
            const auto t0 = std::chrono::steady_clock::now();
            rc = ::allreduce_entry(sb, rb, count, MPI_FLOAT_H, MPI_SUM_H, nullptr);  // this node
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            if (it) best = std::min(best, us);
        }
        if (rc) break;
        w.shm->r[w.rank].tune_us[nc] = best;
        ++nc;
    }
    hipFree(sb);
    hipFree(rb);
    host_barrier();  // every rank's timings are in the control segment
    w.pipe_grid = g0;
    w.pipe_sub = s0;
    w.pipe_rnt = r0;
    if (rc) {
        MV2_ERR("pipe autotune: probe allreduce failed");
        return rc;
    }
    int pick = 0;
    for (int k = 0; k < nc; ++k) {
        double m = 0;
        for (int j = 0; j < w.size; ++j) m = std::max(m, w.shm->r[j].tune_us[k]);
        w.tune_us[k] = m;
        if (m < w.tune_us[pick]) pick = k;
    }
    host_barrier();  // every rank has read every timing
    w.tune_n = nc;
    w.pipe_grid = w.tune_grid[pick];
    w.pipe_sub = w.tune_sub[pick];
    w.pipe_rnt = w.tune_rnt[pick];
    w.pipe_tuned = 1;
    MV2_DEBUG("pipe autotune: grid %d sub %zu %s stores (%.1f us of %d candidates)", w.pipe_grid, w.pipe_sub,
              w.pipe_rnt ? "non-temporal" : "plain", w.tune_us[pick], nc);
    return oneshot_autotune();
}

// The one-shot kernel pushes a rank's whole operand to every peer (n-1 times the link bytes of
// the pipelined kernel) but needs one flag exchange instead of two per round: where it stops
// paying is again a property of the links.  Probe 32 KiB .. the arena slot with both kernels
// (max over ranks) and keep the one-shot path up to the largest size it wins, scanning up.
// The path never changes a result: both kernels evaluate the call's plan.
int oneshot_autotune() {
    World &w = world();
    const int MPI_FLOAT_H = 0x4c00040a, MPI_SUM_H = 0x58000003;
    // probe up to the slot (1 MiB when the node tunes, world.cpp), or to an explicit MV2AMD_ONESHOT_MAX
    const size_t top = getenv("MV2AMD_ONESHOT_MAX") ? std::min(w.oneshot_max, w.slot_bytes) : w.slot_bytes;
    void *sb = nullptr, *rb = nullptr;
    if (top < ((size_t)32 << 10) || hipMalloc(&sb, top) != hipSuccess || hipMalloc(&rb, top) != hipSuccess) {
        if (sb) hipFree(sb);
        return 0;
    }
    hipMemset(sb, 0, top);
    hipDeviceSynchronize();
    const size_t keep = w.oneshot_max;
    size_t sizes[kTuneMax / 2];
    int ns = 0;
    for (size_t b = (size_t)32 << 10; b <= top && ns < kTuneMax / 2; b <<= 1) sizes[ns++] = b;
    int rc = 0;
    for (int i = 0; i < ns && !rc; ++i) {
        for (int path = 0; path < 2 && !rc; ++path) {  // 0: one-shot, 1: pipelined
            w.oneshot_max = path ? 0 : top;  // one-shot up to the probed size, or never
            double best = 1e30;
            for (int it = 0; it < 6 && !rc; ++it) {
                host_barrier();
                const auto t0 = std::chrono::steady_clock::now();
                rc = ::allreduce_entry(sb, rb, sizes[i] / 4, MPI_FLOAT_H, MPI_SUM_H, nullptr);
                const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                if (it) best = std::min(best, us);
            }
            w.shm->r[w.rank].tune_us[2 * i + path] = best;
        }
    }
    hipFree(sb);
    hipFree(rb);
    w.oneshot_max = keep;
    host_barrier();
    if (rc) return rc;
    size_t thr = 0;
    for (int i = 0; i < ns; ++i) {
        double one = 0, pipe = 0;
        for (int j = 0; j < w.size; ++j) {
            one = std::max(one, w.shm->r[j].tune_us[2 * i]);
            pipe = std::max(pipe, w.shm->r[j].tune_us[2 * i + 1]);
        }
        w.os_tune_us[i][0] = one;
        w.os_tune_us[i][1] = pipe;
    }
    for (int i = 0; i < ns && w.os_tune_us[i][0] <= w.os_tune_us[i][1]; ++i) thr = sizes[i];  // wins from the bottom
    host_barrier();
    w.os_tune_n = ns;
    if (thr) w.oneshot_max = thr;  // below 32 KiB the one-shot kernel is kept
    else w.oneshot_max = (size_t)16 << 10;
    MV2_DEBUG("one-shot autotune: one-shot up to %zu bytes", w.oneshot_max);
    return 0;
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
    if (!strcmp(key, "max_grid")) w.max_grid = (int)std::min<long>(std::max(1L, value), kDoneMaxGrid);
    else if (!strcmp(key, "rl_grid")) w.rl_grid = (int)std::min<long>(std::max(1L, value), kDoneMaxGrid);
    else if (!strcmp(key, "rl_tiny_max")) w.rl_tiny_max = (size_t)std::max(0L, value);
    else if (!strcmp(key, "pipe_grid")) w.pipe_grid = (int)value;
    else if (!strcmp(key, "pipe_sub")) w.pipe_sub = (size_t)value;
    else if (!strcmp(key, "light_release")) w.light_release = (int)value;
    else if (!strcmp(key, "withhold_done")) g_withhold_done = (int)value;
    else if (!strcmp(key, "fake_split")) g_fake_split = (int)value;
    else if (!strcmp(key, "oneshot_max")) {
        if ((size_t)value > w.slot_bytes && w.size > 1) return E_ARG;
        w.oneshot_max = (size_t)value;
    } else return E_ARG;
    return 0;
}

int mv2h_get_info(const char *key, long *value) {
    World &w = world();
    if (!key || !value) return E_ARG;
    if (!strcmp(key, "nshare")) *value = w.nshare;
    else if (!strcmp(key, "device")) *value = w.device;
    else if (!strcmp(key, "cus")) *value = w.cus;
    else if (!strcmp(key, "light_release")) *value = w.light_release;
    else if (!strcmp(key, "oneshot_max")) *value = (long)w.oneshot_max;
    else if (!strcmp(key, "nnodes")) *value = w.nnodes;
    else if (!strcmp(key, "node")) *value = w.node;
    else if (!strcmp(key, "pipe_grid")) *value = w.pipe_grid;
    else if (!strcmp(key, "pipe_sub")) *value = (long)w.pipe_sub;
    else if (!strcmp(key, "pipe_tuned")) *value = w.pipe_tuned;
    else if (!strcmp(key, "tune_n")) *value = w.tune_n;
    else if (!strcmp(key, "pipe_rnt")) *value = w.pipe_rnt;
    else if (!strcmp(key, "os_tune_n")) *value = w.os_tune_n;
    else if (!strcmp(key, "init_us")) *value = (long)(w.init_ms * 1e3 + 0.5);
    else if (!strcmp(key, "selftest_us")) *value = (long)(w.selftest_ms * 1e3 + 0.5);
    else if (!strcmp(key, "autotune_us")) *value = (long)(w.tune_ms * 1e3 + 0.5);
    else if (!strcmp(key, "hip_init_us")) *value = (long)(w.hip_init_ms * 1e3 + 0.5);
    else if (!strcmp(key, "code_load_us")) *value = (long)(w.code_load_ms * 1e3 + 0.5);
    else if (!strcmp(key, "selftest_calls")) *value = w.selftest_calls;
    else if (!strcmp(key, "call_allocs")) *value = (long)w.call_allocs;
    else if (!strcmp(key, "pool_trims")) *value = (long)w.pool_trims;
    else if (!strcmp(key, "rl_tiny_max")) *value = (long)w.rl_tiny_max;
    else if (!strcmp(key, "aql_calls")) *value = (long)w.aql_calls;
    else if (!strcmp(key, "aql_kernels")) *value = aql_kernels();
    else if (!strcmp(key, "aql_acquire")) *value = aql_acquire_scope();
    else if (!strcmp(key, "aql_skip_lib")) *value = aql_skips(0);
    else if (!strcmp(key, "aql_skip_null")) *value = aql_skips(1);
    // constants chosen on one shared GPU (not probed at MPI_Init; the N > 1 bench line names them)
    else if (!strcmp(key, "ar_scalar_max")) *value = env_long_coll("MV2AMD_AR_SCALAR_MAX", 1024);
    else if (!strcmp(key, "rs_scalar_max")) *value = env_long_coll("MV2AMD_RS_SCALAR_MAX", 4096);
    else if (!strcmp(key, "p2p_kernel_copy")) {
        const char *v = getenv("MV2AMD_P2P_KERNEL_COPY");
        *value = (v && *v) ? *v != '0' : w.nshare <= 4;
    }
    else if (!strcmp(key, "done_late")) *value = (long)w.done_late;
    else if (!strcmp(key, "done_queried")) *value = (long)w.done_queried;
    else if (!strcmp(key, "done_missed")) *value = (long)w.done_missed;
    else if (!strcmp(key, "done_xcd_split")) *value = (long)w.done_xcd_split;
    else if (!strcmp(key, "p2p_unexpected")) *value = (long)p2p_unexpected_matched();
    else if (!strcmp(key, "hw_queues_set")) *value = w.hw_queues_set;
    else if (!strcmp(key, "uop_in_bytes")) *value = (long)w.uop_in_bytes;
    else if (!strcmp(key, "uop_area_bytes")) *value = (long)w.uop_area_bytes;
    else if (!strcmp(key, "uop_stage_us")) *value = (long)(w.uop_ns[0] / 1000);
    else if (!strcmp(key, "uop_fetch_us")) *value = (long)(w.uop_ns[1] / 1000);
    else if (!strcmp(key, "uop_eval_us")) *value = (long)(w.uop_ns[2] / 1000);
    else if (!strcmp(key, "uop_deliver_us")) *value = (long)(w.uop_ns[3] / 1000);
    else if (!strncmp(key, "os_tune_one_", 12) || !strncmp(key, "os_tune_pipe_", 13)) {
        const long i = strtol(strrchr(key, '_') + 1, nullptr, 10);
        if (i < 0 || i >= w.os_tune_n) return E_ARG;
        *value = (long)(w.os_tune_us[i][key[8] == 'o' ? 0 : 1] + 0.5);
    }
    else if (!strncmp(key, "tune_", 5) && strrchr(key, '_') && strrchr(key, '_')[1]) {
        // tune_grid_<k> / tune_sub_<k> / tune_rnt_<k> / tune_us_<k>: candidate k of pipe_autotune
        char *end = nullptr;
        const long k = strtol(strrchr(key, '_') + 1, &end, 10);
        if (!end || *end || k < 0 || k >= w.tune_n) return E_ARG;
        if (!strncmp(key, "tune_grid_", 10)) *value = w.tune_grid[k];
        else if (!strncmp(key, "tune_sub_", 9)) *value = (long)w.tune_sub[k];
        else if (!strncmp(key, "tune_rnt_", 9)) *value = w.tune_rnt[k];
        else if (!strncmp(key, "tune_us_", 8)) *value = (long)(w.tune_us[k] + 0.5);
        else return E_ARG;
    } else return E_ARG;
    return 0;
}

int mv2h_init(void) { return world_init(); }
int mv2h_finalize(void) { return world_finalize(); }
int mv2h_rank(void) { return world().grank; }
int mv2h_size(void) { return world().gsize; }
int mv2h_local_rank(void) { return world().local_rank; }

int mv2h_barrier(void) { return global_barrier(); }

int mv2h_defer_begin(void) {
    World &w = world();
    w.defer = true;
    w.deferred = 0;
    return 0;
}

int mv2h_defer_end(unsigned long long *ticket) {
    World &w = world();
    w.defer = false;
    if (ticket) *ticket = w.deferred;
    w.deferred = 0;
    return 0;
}

int mv2h_test_ticket(unsigned long long ticket, int *done) {
    World &w = world();
    if (done) *done = 1;
    if (ticket == 0 || !w.done_flag) return 0;
    if (__atomic_load_n(w.done_flag, __ATOMIC_ACQUIRE) < ticket) {
        // the word is the normal path; the stream only once this ticket is 200 us late
        static unsigned long long last_ticket = 0;
        static uint64_t since = 0;
        const uint64_t t = now_ns();
        if (ticket != last_ticket) {
            last_ticket = ticket;
            since = t;
        }
        if (t - since < 200000) {
            if (done) *done = 0;
            return 0;
        }
        const hipError_t q = hipStreamQuery(w.stream);
        if (q == hipErrorNotReady) {
            if (done) *done = 0;
            return 0;
        }
        if (q != hipSuccess) return E_INTERN;
    }
    if (__atomic_load_n(w.done_flag + 1, __ATOMIC_ACQUIRE) > w.split_seen) {
        // the word came from a kernel whose block groups were split over XCDs: done once the
        // stream is (settle_split)
        const hipError_t q = hipStreamQuery(w.stream);
        if (q == hipErrorNotReady) {
            if (done) *done = 0;
            return 0;
        }
        if (q != hipSuccess || settle_split(w.stream) != hipSuccess) return E_INTERN;
    }
    return check_err_word();
}

int mv2h_wait_ticket(unsigned long long ticket) {
    World &w = world();
    if (ticket == 0 || !w.done_flag) return 0;
    const hipError_t e = wait_done(w.stream, ticket);
    if (e != hipSuccess) {
        MV2_ERR("waiting for a nonblocking collective failed: %s", hipGetErrorString(e));
        return E_INTERN;
    }
    return check_err_word();
}

// ---------------------------------------------------------------------------
// part (1): MPI_Reduce_local on device buffers (reduce_local.c:36-173)
// ---------------------------------------------------------------------------
int mv2h_reduce_local(const void *in, void *inout, size_t count, int dtype, int op, void *stream) {
    hp_entry();
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    if (count == 0) return 0;  // reduce_local.c:49
    if ((rc = kind_supported(dt))) return rc;
    if ((rc = ensure_init_for_device())) return rc;
    World &w = world();
    const int oi = op_index(op);
    const size_t bytes = count * (size_t)dt->extent;
    // host buffers: staged through device scratch, reduced on the GPU
    const bool din = is_device(in), dio = is_device(inout);
    // small device operands on the library's stream: the one-wave kernel dispatched straight into
    // the library's HSA queue when nothing of HIP's ordering is pending (runtime/aql.cpp)
    if (din && dio && !stream && oi < OP_REPLACE && bytes <= w.rl_tiny_max && (!w.last_st || w.last_st == w.stream)) {
        const int r = aql_reduce_local(oi, dt->kind, in, inout, count, dt->extent);
        if (r < 0) return -r;
        if (r == 1) {
            ++w.aql_calls;
            return check_err_word();
        }
    }
    hipStream_t st = pick_stream(stream);
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
        cfg.done = arm_done(st);
        cfg.tiny_max = w.rl_tiny_max;
        rc = launch_reduce_local(oi, dt->kind, din_p, dio_p, count, dt->extent, cfg);
    }
    tmark1(st);
    if (rc) return rc;
    if (!dio) enq_copy(inout, dio_p, bytes, st);
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
    LaunchCfg cfg{std::min(world().rl_grid, 4096), 2, st};
    tmark0(st);
    rc = launch_reduce_n(oi, dt->kind, srcs, nsrc, dst, count, dt->extent, tp, cfg);
    tmark1(st);
    if (rc) return rc;
    return finish(st, world().timing);
}

static_assert(sizeof(mv2h_progset) == sizeof(ProgSet), "mv2h_progset mirrors ProgSet");

int mv2h_reduce_n_prog(const void *const *srcs, int nsrc, void *dst, size_t count, int dtype, int op,
                       const mv2h_progset *ps, void *stream) {
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    if ((rc = kind_supported(dt))) return rc;
    if (nsrc < 1 || nsrc > kMaxRanks || !ps || ps->nprog < 1 || ps->nprog > kMaxRanks || ps->blk == 0) return E_ARG;
    for (int b = 0; b < ps->nprog; ++b) {
        const mv2h_prog &p = ps->p[b];
        if (p.nsteps > kMaxRanks - 1 || p.res >= nsrc) return E_ARG;
        for (int i = 0; i < p.nsteps; ++i)
            if (p.dst[i] >= nsrc || p.src[i] >= nsrc) return E_ARG;
    }
    if (count == 0) return 0;
    if ((rc = ensure_init_for_device())) return rc;
    const int oi = op_index(op);
    if (oi >= OP_REPLACE) return E_OP;
    hipStream_t st = pick_stream(stream);
    TreeParams tp = tree_base(nsrc);
    tp.linear = 4;
    memcpy(&tp.ps, ps, sizeof(ProgSet));
    LaunchCfg cfg{std::min(world().rl_grid, 4096), 2, st};
    tmark0(st);
    rc = launch_reduce_n(oi, dt->kind, srcs, nsrc, dst, count, dt->extent, tp, cfg);
    tmark1(st);
    if (rc) return rc;
    return finish(st, world().timing);
}

int mv2h_reduce_scatter_table(int n, long nbytes) { return reduce_scatter_table(n, nbytes); }

int mv2h_mn_allreduce_table(int ppn, int gsize, long nbytes, int *intra, int *inter) {
    int in = -1, it = -1;
    const int t = mn_allreduce_table(ppn, gsize, nbytes, &in, &it);
    if (intra) *intra = t == 0 ? in : -1;
    if (inter) *inter = t == 0 ? it : -1;
    return t;
}

int mv2h_nbc_begin(int kind) {
    if (kind < MV2H_NBC_NONE || kind > MV2H_NBC_IREDUCE_SCATTER_BLOCK) return E_ARG;
    nbc_set(kind);
    return 0;
}
int mv2h_nbc_end(void) {
    nbc_set(NBC_NONE);
    return 0;
}

int mv2h_knobs_reload(void) {
    knobs_reload();
    return 0;
}

int mv2h_set_topology(int nlevels, const int *colors, int n) {
    if (nlevels < 0 || nlevels > kTopoLevels || n < 0 || n > kMaxRanks || (nlevels && !colors)) return E_ARG;
    Topo t{};
    t.nlevels = nlevels;
    for (int l = 0; l < nlevels; ++l)
        for (int r = 0; r < n; ++r) t.color[l][r] = colors[l * n + r];
    topo_set(t);
    return 0;
}

int mv2h_get_topology(int *nlevels, int *colors, int n) {
    if (!nlevels || n < 0 || n > kMaxRanks) return E_ARG;
    const Topo &t = topo();
    *nlevels = t.nlevels;
    if (colors)
        for (int l = 0; l < t.nlevels; ++l)
            for (int r = 0; r < n; ++r) colors[l * n + r] = t.color[l][r];
    return 0;
}

int mv2h_plan(int coll, int n, int rank, int root, size_t count, const size_t *counts, int dtype, int opkind,
              int in_place, int *algo, int *inner, int *unpinned, mv2h_progset *ps) {
    const DtypeInfo *dt = dtype_lookup(dtype);
    if (!dt) return E_TYPE;
    if (n < 1 || n > kMaxRanks || rank < 0 || rank >= n || opkind < 0 || opkind > 2) return E_ARG;
    Plan p;
    int rc;
    switch (coll) {
    case MV2H_COLL_ALLREDUCE:
        rc = plan_allreduce(n, rank, count, dt->size, dt->extent, in_place != 0, 0, &p, opkind);
        break;
    case MV2H_COLL_ALLREDUCE_RS:
        rc = plan_allreduce(n, rank, count, dt->size, dt->extent, in_place != 0, ALG_PT2PT_RS, &p, opkind);
        break;
    case MV2H_COLL_REDUCE:
        if (root < 0 || root >= n) return E_ROOT;
        rc = plan_reduce(n, rank, root, count, dt->size, dt->extent, &p, opkind);
        break;
    case MV2H_COLL_REDUCE_SCATTER:
        if (!counts) return E_ARG;
        rc = plan_reduce_scatter(n, rank, counts, dt->size, dt->extent, &p, opkind);
        break;
    default: return E_ARG;
    }
    if (rc) return rc;
    if (algo) *algo = p.algo;
    if (inner) *inner = p.inner;
    if (unpinned) *unpinned = p.unpinned;
    if (ps) memcpy(ps, &p.ps, sizeof(ProgSet));
    return 0;
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

// Device staging space of a call.  A captured call (graph lane) cannot use the shared scratch
// buffers — a graph keeps their addresses for every replay while later calls regrow or reuse
// them — so it takes a private piece of a pool that lives until MPI_Finalize.
static void *call_scratch(int idx, size_t bytes) {
    World &w = world();
    if (!w.graph) return get_scratch(idx, bytes);
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (!w.g_pool || w.g_pool_used + need > w.g_pool_bytes) {
        MV2_ERR("graph lane: staging pool exhausted (%zu bytes)", w.g_pool_bytes);
        return nullptr;
    }
    void *p = w.g_pool + w.g_pool_used;
    w.g_pool_used += need;
    return p;
}

static int stage_in(const void *send, void *recv, size_t sbytes, size_t rbytes, bool in_place, hipStream_t st,
                    Staged &s) {
    s.copy_back = false;
    s.user_recv = recv;
    s.bytes = rbytes;
    const bool recv_ok = is_device(recv) && ((uintptr_t)recv % 16 == 0);
    beacon(BC_STAGE);
    if (recv_ok) {
        s.recv = (char *)recv;
    } else {
        s.recv = (char *)call_scratch(1, rbytes);
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
            char *t = (char *)call_scratch(0, sbytes);
            if (!t) return E_NO_MEM;
            hipMemcpyAsync(t, send, sbytes, hipMemcpyDefault, st);
            s.send = t;
        }
    }
    return 0;
}

// the staged result copied back to the caller's buffer; E_INTERN when the copy cannot be
// enqueued (the call must then fail rather than return with the result never delivered)
static int stage_out(const Staged &s, hipStream_t st) {
    if (s.copy_back && enq_copy_last(s.user_recv, s.recv, s.bytes, st) != hipSuccess) return E_INTERN;
    return 0;
}

// One allreduce over `count` elements in the order `tp` (ring = true: the flat
// ring's chunking, segment j = ring chunk j; count is a multiple of n).
static int allreduce_impl(const void *sendbuf, void *recvbuf, size_t count, const DtypeInfo *dt, int oi,
                          hipStream_t st, const TreeParams &tp_in, bool ring = false) {
    World &w = world();
    const size_t bytes = count * (size_t)dt->extent;
    const bool in_place = sendbuf == (const void *)-1 || sendbuf == recvbuf;
    Staged s;
    int rc = stage_in(sendbuf, recvbuf, bytes, bytes, in_place, st, s);
    if (rc) return rc;
    const int n = w.size;
    if (n == 1 || oi == OP_NO_OP) {
        if (!in_place && oi != OP_NO_OP) hipMemcpyAsync(s.recv, s.send, bytes, hipMemcpyDeviceToDevice, st);
        if ((rc = stage_out(s, st))) return rc;
        return finish(st, false);
    }
    if (oi == OP_REPLACE) {
        // result of REPLACE over ranks 0..n-1 in rank order: rank n-1's data; take the two-level
        // linear chain semantics: recv = x_{n-1} everywhere.  Realised as a broadcast from n-1.
        if (!in_place) hipMemcpyAsync(s.recv, s.send, bytes, hipMemcpyDeviceToDevice, st);
        if ((rc = stage_out(s, st))) return rc;
        rc = finish(st, false);
        if (rc) return rc;
        return mv2h_bcast(recvbuf, bytes, n - 1, nullptr);
    }
    TreeParams tp = tp_in;
    const size_t nvec = bytes / 16;
    const int gcap = grid_cap();
    if (!ring && bytes <= w.oneshot_max && bytes <= w.slot_bytes) {
        // the degree-d tree (the default small-message order at 6-8 ranks) on its own evaluator
        if (tp.linear == 4) {
            const int d = progs_grouped(tp.ps, n);
            if (d) {
                tp.linear = 5;
                tp.pof2 = d;
            }
        }
        OneShotArgs a{};
        oneshot_common(a, st);
        a.send = s.send;
        a.recv = s.recv;
        a.count = count;
        // small operands element by element in one workgroup, on the compact kernel whose code
        // holds no vector phases (kernels_impl.h LOneShot: 8 B launch -> completion 8.8 -> 7.8 us
        // at 2 shared ranks, profiles/r05az; the general kernel's element-wise body measured no
        // faster than its vector body, r05z)
        static const long scalar_max = env_long_coll("MV2AMD_AR_SCALAR_MAX", 1024);
        const size_t nv = bytes <= (size_t)scalar_max ? 0 : nvec;
        a.nvec = nv;
        a.tp = tp;
        const int g = oneshot_grid(nv, gcap);
        LaunchCfg cfg = coll_cfg(g, st);
        tmark0(st);
        rc = launch_oneshot(oi, dt->kind, a, dt->extent, cfg);
        tmark1(st);
        if (rc) return rc;
        if ((rc = stage_out(s, st))) return rc;
        return finish(st, w.timing);
    }
    // pipelined direct reduce-scatter + all-gather, pushed through the arenas
    PipeArgs a{};
    a.mode = PIPE_AR;
    a.send = s.send;
    a.recv = s.recv;
    a.esize = dt->extent;
    if (ring) {
        // segment j = ring chunk j.  Chunks that are not 16-byte multiples keep their
        // misalignment through the arena slots (coll/pipe.h: scalar head, aligned body);
        // only operands whose base is not 16-byte aligned go through padded copies
        tp.linear = 3;
        const size_t cb = (count / n) * (size_t)dt->extent;
        if (cb % 16 == 0 || ((uintptr_t)s.send % 16 == 0 && (uintptr_t)s.recv % 16 == 0)) {
            for (int j = 0; j < n; ++j) {
                a.seg_off[j] = a.recv_off[j] = (size_t)j * cb;
                a.seg_len[j] = cb;
            }
        } else {
            const size_t pcb = (cb + 15) & ~(size_t)15;
            char *ps = (char *)call_scratch(3, pcb * n), *pr = (char *)call_scratch(4, pcb * n);
            if (!ps || !pr) return E_NO_MEM;
            if (hipMemcpy2DAsync(ps, pcb, s.send, cb, cb, n, hipMemcpyDeviceToDevice, st) != hipSuccess)
                return E_INTERN;
            for (int j = 0; j < n; ++j) {
                a.seg_off[j] = a.recv_off[j] = (size_t)j * pcb;
                a.seg_len[j] = cb;
            }
            a.send = ps;
            a.recv = pr;
            a.tp = tp;
            if ((rc = run_pipe(a, oi, dt, st))) return rc;
            if (hipMemcpy2DAsync(s.recv, cb, pr, pcb, cb, n, hipMemcpyDeviceToDevice, st) != hipSuccess)
                return E_INTERN;
            world().pending = 0;
            if ((rc = stage_out(s, st))) return rc;
            return finish(st, w.timing);
        }
    } else {
        even_segments(a, bytes, n);
    }
    a.tp = tp;
    if ((rc = run_pipe(a, oi, dt, st))) return rc;
    if ((rc = stage_out(s, st))) return rc;
    return finish(st, w.timing);
}

// MPIR_Allreduce_index_tuned_intra_MV2's one-node choice (orders.cpp
// plan_allreduce).  The ring wrapper (allreduce_osu.c:3758-3818) runs the
// ring over the first (count/n)*n elements and pt2pt_rs over the remainder;
// with MPI_IN_PLACE the ring body itself falls back to pt2pt_rs (:4095-4100),
// still over the two ranges separately; count < n leaves the ring nothing.
static int allreduce_select(const void *sendbuf, void *recvbuf, size_t count, const DtypeInfo *dt, int oi,
                            hipStream_t st) {
    World &w = world();
    const int n = w.size, me = w.rank;
    const bool reducing = n > 1 && oi != OP_NO_OP && oi != OP_REPLACE;
    const bool in_place = sendbuf == (const void *)-1;
    Plan p;
    if (!reducing) return allreduce_impl(sendbuf, recvbuf, count, dt, oi, st, tree_base(n));
    int rc = plan_allreduce(n, me, count, dt->size, dt->extent, in_place, 0, &p);
    if (rc) return rc;
    log_plan("allreduce", p, count);
    pvar_note(PV_COLL_ALLREDUCE, p, in_place, count, n);
    if (p.algo != ALG_RING) return allreduce_impl(sendbuf, recvbuf, count, dt, oi, st, tree_from_plan(p, n, count, me));
    if (count < (size_t)n) return allreduce_impl(sendbuf, recvbuf, count, dt, oi, st, tree_rs(n, count, me, false));
    const size_t main = (count / n) * n, rest = count - main, off = main * (size_t)dt->extent;
    rc = in_place ? allreduce_impl(sendbuf, recvbuf, main, dt, oi, st, tree_rs(n, main, me, false))
                  : allreduce_impl(sendbuf, recvbuf, main, dt, oi, st, tree_base(n), true);
    if (rc || !rest) return rc;
    return allreduce_impl(in_place ? sendbuf : (const char *)sendbuf + off, (char *)recvbuf + off, rest, dt, oi, st,
                          tree_rs(n, rest, me, false));
}
static int allreduce_entry(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream) {
    hp_entry();
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    if (count == 0) return 0;  // allreduce_osu.c:3730
    if ((rc = kind_supported(dt))) return rc;
    if ((rc = require_world())) return rc;
    return allreduce_select(sendbuf, recvbuf, count, dt, op_index(op), pick_stream(stream));
}
// A stream-ordered call across nodes (MPIX_*_enqueue): the leaders' steps are host-driven, so the
// call waits for the caller's stream, then runs as the blocking call and returns complete; work
// queued on the stream afterwards sees the result.  Stream order without the overlap (graph
// capture stays refused, enqueue_checks).  The EnqueueScope of the entry point clears the flag.
static int mn_stream_order(void **stream) {
    if (hipStreamSynchronize((hipStream_t)*stream) != hipSuccess) return E_INTERN;
    world().enqueue = false;
    *stream = nullptr;
    return 0;
}
static int mn_allreduce(const void *, void *, size_t, int, int, void *);
static int mn_reduce(const void *, void *, size_t, int, int, int, void *);
// A nonblocking collective across nodes completes at initiation (MPI allows it: the request is
// complete when MPI_Wait / MPI_Test first sees it); the node steps inside run blocking.
struct MnBlocking {
    bool was;
    MnBlocking() : was(world().defer) { world().defer = false; }
    ~MnBlocking() {
        world().defer = was;
        world().deferred = 0;
    }
};

static int mn_reduce_scatter(const void *, void *, const size_t *, int, int, void *);

int mv2h_allreduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream) {
    if (world().nnodes > 1) {
        int rc0 = 0;
        if (world().enqueue && (rc0 = mn_stream_order(&stream))) return rc0;
        MnBlocking nb;
        pvar_begin();
        const int rc = mn_allreduce(sendbuf, recvbuf, count, dtype, op, stream);
        pvar_end(rc == 0);
        return rc;
    }
    pvar_begin();
    const int rc = allreduce_entry(sendbuf, recvbuf, count, dtype, op, stream);
    pvar_end(rc == 0);
    return rc;
}

// forced: the programs to run instead of the one-node selection's (a node step of
// MPIR_Reduce_two_level_helper_MV2 across nodes, whose function the multi-node table names)
static int reduce_entry(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, int root, void *stream,
                        const Plan *forced = nullptr) {
    hp_entry();
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
    const int oi = op_index(op);
    const bool is_root = w.rank == root;
    const bool in_place = sendbuf == (const void *)-1 || (is_root && sendbuf == recvbuf);
    // MPIR_Reduce_index_tuned_intra_MV2's one-node choice (orders.cpp plan_reduce)
    Plan p;
    if (forced) p = *forced;
    else if ((rc = plan_reduce(w.size, w.rank, root, count, dt->size, dt->extent, &p))) return rc;
    log_plan("reduce", p, count);
    pvar_note(PV_COLL_REDUCE, p, in_place, count, w.size);
    const TreeParams tp = tree_from_plan(p, w.size, count, w.rank);
    // small messages, REPLACE / NO_OP, one rank: every rank computes the root's result
    // (one-shot); non-roots discard theirs
    if (w.size == 1 || oi >= OP_REPLACE || (bytes <= w.oneshot_max && bytes <= w.slot_bytes)) {
        if (is_root) return allreduce_impl(sendbuf, recvbuf, count, dt, oi, st, tp);
        void *tmp = call_scratch(2, bytes);
        if (!tmp) return E_NO_MEM;
        return allreduce_impl(in_place ? recvbuf : sendbuf, tmp, count, dt, oi, st, tp);
    }
    // pipelined: scatter -> reduce -> push to the root -> root gathers
    Staged s{};
    if (is_root) {
        if ((rc = stage_in(sendbuf, recvbuf, bytes, bytes, in_place, st, s))) return rc;
    } else {
        s.recv = nullptr;
        s.copy_back = false;
        const void *src = in_place ? recvbuf : sendbuf;
        if (is_device(src) && (uintptr_t)src % 16 == 0) {
            s.send = (const char *)src;
        } else {
            char *t = (char *)call_scratch(0, bytes);
            if (!t) return E_NO_MEM;
            hipMemcpyAsync(t, src, bytes, hipMemcpyDefault, st);
            s.send = t;
        }
    }
    PipeArgs a{};
    a.mode = PIPE_RED;
    a.root = root;
    a.send = s.send;
    a.recv = s.recv;
    a.esize = dt->extent;
    a.tp = tp;
    even_segments(a, bytes, w.size);
    if ((rc = run_pipe(a, oi, dt, st))) return rc;
    if (is_root && (rc = stage_out(s, st))) return rc;
    return finish(st, w.timing);
}
int mv2h_reduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, int root, void *stream) {
    if (world().nnodes > 1) {
        int rc0 = 0;
        if (world().enqueue && (rc0 = mn_stream_order(&stream))) return rc0;
        MnBlocking nb;
        pvar_begin();
        const int rc = mn_reduce(sendbuf, recvbuf, count, dtype, op, root, stream);
        pvar_end(rc == 0);
        return rc;
    }
    pvar_begin();
    const int rc = reduce_entry(sendbuf, recvbuf, count, dtype, op, root, stream);
    pvar_end(rc == 0);
    return rc;
}

static int reduce_scatter_entry(const void *sendbuf, void *recvbuf, const size_t *recvcounts, int dtype, int op,
                        void *stream) {
    hp_entry();
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    if ((rc = kind_supported(dt))) return rc;
    if ((rc = require_world())) return rc;
    World &w = world();
    const int n = w.size;
    const size_t ext = dt->extent;
    size_t total = 0, off = 0, padded = 0;
    bool natural = true;  // every segment starts 16-byte aligned in the caller's layout
    for (int j = 0; j < n; ++j) {
        if (j == w.rank) off = total;
        if ((total * ext) % 16) natural = false;
        total += recvcounts[j];
        padded += (recvcounts[j] * ext + 15) & ~(size_t)15;
    }
    if (total == 0) return 0;
    const int oi = op_index(op);
    hipStream_t st = pick_stream(stream);
    const size_t mycnt = recvcounts[w.rank];
    const bool in_place = sendbuf == (const void *)-1;
    const void *send = in_place ? recvbuf : sendbuf;
    if (n == 1 || oi == OP_NO_OP || oi == OP_REPLACE) {
        if (!in_place && oi != OP_NO_OP && mycnt)
            hipMemcpyAsync(recvbuf, (const char *)send + off * ext, mycnt * ext, hipMemcpyDefault, st);
        return finish(st, false);
    }
    // small messages: the one-shot reduce-scatter (each peer pushed only its own block, one flag
    // exchange, this rank's block reduced in program order) when the operand fits an arena slot,
    // every block starts on a 16-byte boundary and the algorithm is not the ring (whose rotated
    // chain only the pipelined kernel evaluates).  Only the counts, the type and the plan enter
    // the choice, so every rank makes it alike.
    Plan p;
    if ((rc = plan_reduce_scatter(n, w.rank, recvcounts, dt->size, dt->extent, &p))) return rc;
    // Blocks off 16-byte boundaries take the same kernel element by element when the whole operand
    // is small (kOneShotScalar; osu_reduce_scatter 8 B at 2 shared ranks: 16.4 us pipelined).
    constexpr size_t kOneShotScalar = 2048;
    bool os = !in_place && p.algo != ALG_RS_RING && (size_t)dt->size == ext && 16 % ext == 0 &&
              total * ext <= std::min(w.oneshot_max, w.slot_bytes);
    bool aligned = true;
    for (size_t j = 0, off0 = 0; j < (size_t)n; off0 += recvcounts[j], ++j) aligned = aligned && (off0 * ext) % 16 == 0;
    if (!aligned && total * ext > kOneShotScalar) os = false;
    // small operands element by element even when aligned: 1.9 / 2.3 us faster at 2 / 4 shared
    // ranks from 32 B to 4 KiB than the vector body (profiles/r05y)
    static const long scalar_max = env_long_coll("MV2AMD_RS_SCALAR_MAX", 4096);
    if (total * ext <= (size_t)scalar_max) aligned = false;
    if (os) {
        log_plan("reduce_scatter", p, total);
        pvar_note(PV_COLL_REDUCE_SCATTER, p, false, total, n);
        const char *src = (const char *)send;
        if (!is_device(send) || (uintptr_t)send % 16) {
            char *t = (char *)call_scratch(0, total * ext);
            if (!t) return E_NO_MEM;
            beacon(BC_STAGE);
            hipMemcpyAsync(t, send, total * ext, hipMemcpyDefault, st);
            src = t;
        }
        const bool direct = is_device(recvbuf) && (uintptr_t)recvbuf % 16 == 0;
        char *dst = (char *)recvbuf;
        if (!direct && mycnt && !(dst = (char *)call_scratch(1, mycnt * ext))) return E_NO_MEM;
        OneShotArgs o{};
        oneshot_common(o, st);
        o.send = src;
        o.recv = dst;
        o.count = total;
        o.nvec = aligned ? total * ext / 16 : 0;
        o.rs = 1;
        size_t vmax = 0;
        for (size_t j = 0, e = 0; j < (size_t)n; e += recvcounts[j], ++j) {
            o.wlo[j] = e;
            o.wcnt[j] = recvcounts[j];
            vmax = std::max(vmax, (recvcounts[j] * ext + 15) / 16);
        }
        TreeParams tp = tree_base(n);
        tp.linear = 4;
        tp.ps = p.ps;
        o.tp = tp;
        LaunchCfg cfg = coll_cfg(oneshot_grid(aligned ? vmax : 0, grid_cap()), st);
        tmark0(st);
        rc = launch_oneshot(oi, dt->kind, o, dt->extent, cfg);
        tmark1(st);
        if (rc) return rc;
        if (!direct && mycnt && enq_copy_last(recvbuf, dst, mycnt * ext, st) != hipSuccess) return E_INTERN;
        return finish(st, w.timing);
    }
    PipeArgs a{};
    a.mode = PIPE_RS;
    a.esize = (int)ext;
    // operand: the caller's buffer when it is aligned device memory (and not IN_PLACE:
    // the result overwrites the operand's head) — segments off 16-byte boundaries keep
    // their misalignment through the kernel; otherwise a staged copy with every segment
    // padded to 16 bytes
    (void)natural;
    if (!in_place && is_device(send) && (uintptr_t)send % 16 == 0) {
        a.send = (const char *)send;
        size_t o = 0;
        for (int j = 0; j < n; ++j) {
            a.seg_off[j] = o * ext;
            a.seg_len[j] = recvcounts[j] * ext;
            o += recvcounts[j];
        }
    } else {
        char *t = (char *)call_scratch(0, padded);
        if (!t) return E_NO_MEM;
        beacon(BC_STAGE);
        size_t o = 0, po = 0;
        for (int j = 0; j < n; ++j) {
            const size_t len = recvcounts[j] * ext;
            if (len) hipMemcpyAsync(t + po, (const char *)send + o * ext, len, hipMemcpyDefault, st);
            a.seg_off[j] = po;
            a.seg_len[j] = len;
            o += recvcounts[j];
            po += (len + 15) & ~(size_t)15;
        }
        a.send = t;
    }
    // the result must share my segment's misalignment: the caller's buffer when it does,
    // else a scratch block at that misalignment, copied out after the kernel
    const size_t mis = a.seg_off[w.rank] & 15;
    const bool direct = is_device(recvbuf) && (uintptr_t)recvbuf % 16 == mis;
    char *dst = (char *)recvbuf;
    a.recv_off[w.rank] = 0;
    if (!direct && mycnt) {
        char *t = (char *)call_scratch(1, mycnt * ext + 16);
        if (!t) return E_NO_MEM;
        dst = t + mis;
    }
    a.recv = dst - (direct ? 0 : mis);
    a.recv_off[w.rank] = direct ? 0 : mis;
    // MPIR_Reduce_scatter_MV2's one-node choice (orders.cpp plan_reduce_scatter): ring,
    // recursive halving, pairwise or reduce + scatter, each in its own order
    log_plan("reduce_scatter", p, total);
    pvar_note(PV_COLL_REDUCE_SCATTER, p, false, total, n);
    TreeParams tp = tree_base(n);
    if (p.algo == ALG_RS_RING) {
        tp.linear = 2;  // rotated sources, specialised chain (coll/pipe.h reduce_round)
    } else {
        tp.linear = 4;
        tp.ps = p.ps;
        a.eshift = (int64_t)off - (int64_t)(a.seg_off[w.rank] / ext);
    }
    a.tp = tp;
    if ((rc = run_pipe(a, oi, dt, st))) return rc;
    if (!direct && mycnt && enq_copy_last(recvbuf, dst, mycnt * ext, st) != hipSuccess) return E_INTERN;
    return finish(st, w.timing);
}
int mv2h_reduce_scatter(const void *sendbuf, void *recvbuf, const size_t *recvcounts, int dtype, int op,
                        void *stream) {
    if (world().nnodes > 1) {
        int rc0 = 0;
        if (world().enqueue && (rc0 = mn_stream_order(&stream))) return rc0;
        MnBlocking nb;
        pvar_begin();
        const int rc = mn_reduce_scatter(sendbuf, recvbuf, recvcounts, dtype, op, stream);
        pvar_end(rc == 0);
        return rc;
    }
    pvar_begin();
    const int rc = reduce_scatter_entry(sendbuf, recvbuf, recvcounts, dtype, op, stream);
    pvar_end(rc == 0);
    return rc;
}

static int allgather_node(const void *sendbuf, void *recvbuf, size_t bytes, void *stream) {
    hp_entry();
    int rc;
    if ((rc = require_world())) return rc;
    if (bytes == 0) return 0;
    World &w = world();
    hipStream_t st = pick_stream(stream);
    const int n = w.size;
    const int me = w.rank;
    const bool in_place = sendbuf == (const void *)-1;
    // direct: rank j's block lands at recvbuf + j*bytes even when that is off a 16-byte
    // boundary (coll/pipe.h keeps each block's misalignment through the slots); the
    // contribution must then share its block's misalignment
    const bool direct = is_device(recvbuf) && (uintptr_t)recvbuf % 16 == 0;
    const size_t pitch = direct ? bytes : (bytes + 15) & ~(size_t)15;
    char *dst = direct ? (char *)recvbuf : (char *)call_scratch(1, pitch * n);
    if (!dst) return E_NO_MEM;
    const char *src = in_place ? (const char *)recvbuf + (size_t)me * bytes : (const char *)sendbuf;
    if (n == 1) {
        if (!in_place) hipMemcpyAsync(recvbuf, src, bytes, hipMemcpyDefault, st);
        return finish(st, false);
    }
    // small blocks: the one-shot kernel (one flag exchange; the choice reads only the size and the
    // node's shared limits, so every rank makes it alike).  Whole 16-byte vectors move as vectors;
    // a block of up to kOneShotBytewise bytes of any other size moves byte by byte (osu_allgather
    // 8 B at 2 shared ranks: 15.6 us through the pipelined kernel)
    constexpr size_t kOneShotBytewise = 2048;
    const bool vec = bytes % 16 == 0;
    if ((vec || bytes <= kOneShotBytewise) && bytes <= std::min(w.oneshot_max, w.slot_bytes)) {
        char *od = direct ? (char *)recvbuf : (char *)call_scratch(1, bytes * n);
        if (!od) return E_NO_MEM;
        const char *os = in_place ? od + (size_t)me * bytes : (const char *)sendbuf;
        if (in_place && !direct) {
            hipMemcpyAsync(od + (size_t)me * bytes, (const char *)recvbuf + (size_t)me * bytes, bytes, hipMemcpyDefault, st);
        } else if (!in_place && !(is_device(sendbuf) && (!vec || (uintptr_t)sendbuf % 16 == 0))) {
            char *t = (char *)call_scratch(0, bytes);
            if (!t) return E_NO_MEM;
            hipMemcpyAsync(t, sendbuf, bytes, hipMemcpyDefault, st);
            os = t;
        }
        OneShotArgs a{};
        oneshot_common(a, st);
        a.mv = 1;
        a.send = os;
        a.recv = od;
        a.count = bytes;
        a.nvec = vec ? bytes / 16 : 0;
        a.pitch = bytes;
        LaunchCfg cfg = coll_cfg(oneshot_grid(a.nvec, grid_cap()), st);
        tmark0(st);
        rc = launch_oneshot_mv(a, cfg);
        tmark1(st);
        if (rc) return rc;
        if (!direct && enq_copy_last(recvbuf, od, bytes * n, st) != hipSuccess) return E_INTERN;
        return finish(st, w.timing);
    }
    const size_t mis = ((size_t)me * pitch) & 15;
    if (!(direct && in_place) && !(is_device(src) && (uintptr_t)src % 16 == mis)) {
        char *t = (char *)call_scratch(0, bytes + 16);
        if (!t) return E_NO_MEM;
        hipMemcpyAsync(t + mis, src, bytes, hipMemcpyDefault, st);
        src = t + mis;
    }
    PipeArgs a{};
    a.mode = PIPE_AG;
    a.send = src;
    a.recv = dst;
    a.esize = 1;
    for (int j = 0; j < n; ++j) {
        a.seg_len[j] = bytes;
        a.recv_off[j] = a.seg_off[j] = (size_t)j * pitch;  // seg_off: the block's misalignment
    }
    if ((rc = run_pipe(a, 0, nullptr, st))) return rc;
    if (!direct) {
        w.pending = 0;
        hipMemcpy2DAsync(recvbuf, bytes, dst, pitch, bytes, n, hipMemcpyDefault, st);
    }
    return finish(st, w.timing);
}

static int bcast_node(void *buffer, size_t bytes, int root, void *stream) {
    hp_entry();
    int rc;
    if ((rc = require_world())) return rc;
    if (bytes == 0) return 0;
    World &w = world();
    if (root < 0 || root >= w.size) return E_ROOT;
    if (w.size == 1) return 0;
    hipStream_t st = pick_stream(stream);
    char *buf = (char *)buffer;
    const bool direct = is_device(buffer) && (uintptr_t)buffer % 16 == 0;
    if (!direct) {
        buf = (char *)call_scratch(1, bytes);
        if (!buf) return E_NO_MEM;
        if (w.rank == root) hipMemcpyAsync(buf, buffer, bytes, hipMemcpyDefault, st);
    }
    // small messages: the one-shot kernel (the root pushes its buffer into every peer's arena slot,
    // one flag exchange); the choice reads only the size and the node's shared limits
    if (bytes <= std::min(w.oneshot_max, w.slot_bytes)) {
        OneShotArgs a{};
        oneshot_common(a, st);
        a.mv = 2;
        a.root = root;
        a.send = buf;
        a.recv = buf;
        a.count = bytes;
        a.nvec = bytes / 16;
        LaunchCfg cfg = coll_cfg(oneshot_grid(a.nvec, grid_cap()), st);
        tmark0(st);
        rc = launch_oneshot_mv(a, cfg);
        tmark1(st);
        if (rc) return rc;
        if (!direct && w.rank != root && enq_copy_last(buffer, buf, bytes, st) != hipSuccess) return E_INTERN;
        return finish(st, w.timing);
    }
    PipeArgs a{};
    a.mode = PIPE_BC;
    a.root = root;
    a.send = buf;
    a.recv = buf;
    a.esize = 1;
    even_segments(a, bytes, w.size);
    if ((rc = run_pipe(a, 0, nullptr, st))) return rc;
    if (!direct && w.rank != root && enq_copy_last(buffer, buf, bytes, st) != hipSuccess) return E_INTERN;
    return finish(st, w.timing);
}

// ---------------------------------------------------------------------------
// Several nodes: MVAPICH2's two-level structure, node step on the
// device kernels above (this process's world is its node), inter-node step between the
// node leaders (local rank 0) over internode.cpp's links with host staging; every
// reduction stays a device kernel (mv2h_reduce_local: the reference's uop(tmp, recv)).
//   Allreduce = MPIR_Allreduce_two_level_MV2 (allreduce_osu.c:1687): node reduction
//     (the node's own allreduce: the degree-4 tree up to 2 KiB / shmem LINEAR, the
//     reference's intra step of its topology-aware and skip-small paths, :2272, :118-160),
//     recursive doubling among the leaders (MPIR_Allreduce_pt2pt_rd_MV2 :360-630, the
//     inter step of both paths, :2215-2262), node broadcast.
//   Bcast = node broadcast at the root's node, binomial over the leaders, node broadcast.
//   Reduce = node reduce to the leader, binomial reduce over the leaders to the root's node
//     (MPIR_Reduce_binomial_MV2 reduce_osu.c:425, commutative form), leader -> root.
//   Allgather = node allgather into the node's section, ring over the leaders, node bcast.
// ---------------------------------------------------------------------------
namespace {
struct MnBufs {
    char *h0 = nullptr, *h1 = nullptr;  // pinned host staging
    size_t hcap = 0;
    char *d0 = nullptr, *d1 = nullptr;  // device: leader partial / received operand
    size_t dcap = 0;
};
MnBufs g_mn;

// host staging h0 / h1 (node leaders: the inter-node messages) and device d0 / d1
int mn_reserve_host(size_t bytes) {
    if (bytes > g_mn.hcap) {
        if (g_mn.h0) hipHostFree(g_mn.h0);
        if (g_mn.h1) hipHostFree(g_mn.h1);
        g_mn.h0 = g_mn.h1 = nullptr;
        g_mn.hcap = 0;
        if (hipHostMalloc((void **)&g_mn.h0, bytes, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&g_mn.h1, bytes, hipHostMallocDefault) != hipSuccess)
            return E_NO_MEM;
        g_mn.hcap = bytes;
    }
    return 0;
}
int mn_reserve_dev(size_t bytes) {
    if (bytes > g_mn.dcap) {
        hipDeviceSynchronize();
        if (g_mn.d0) hipFree(g_mn.d0);
        if (g_mn.d1) hipFree(g_mn.d1);
        g_mn.d0 = g_mn.d1 = nullptr;
        g_mn.dcap = 0;
        if (hipMalloc((void **)&g_mn.d0, bytes) != hipSuccess || hipMalloc((void **)&g_mn.d1, bytes) != hipSuccess)
            return E_NO_MEM;
        g_mn.dcap = bytes;
    }
    return 0;
}
int mn_reserve(size_t bytes) {
    const int rc = mn_reserve_host(bytes);
    return rc ? rc : mn_reserve_dev(bytes);
}

int mn_d2h(void *h, const void *d, size_t b) { return hipMemcpy(h, d, b, hipMemcpyDefault) == hipSuccess ? 0 : E_INTERN; }
int mn_h2d(void *d, const void *h, size_t b) { return hipMemcpy(d, h, b, hipMemcpyDefault) == hipSuccess ? 0 : E_INTERN; }

// The message schedules of MPIR_Allreduce_pt2pt_rd_MV2 (allreduce_osu.c:455-600) and
// MPIR_Allreduce_pt2pt_rs_MV2 (:740-1054: recursive doubling for count < pof2, :802) run as
// messages over n ranks, this one `rank`.  acc (device, count elements of ext bytes) holds the
// operand and ends with the result; tmp (device, as large) receives.  x.xchg(peer, sb, sbytes, rb,
// rbytes) sends and receives (either side may be empty).  Every uop(tmp, recvbuf) is one device
// Reduce_local; builtin ops only (commutative, so recursive doubling never swaps its operands).
struct Xport {
    // send sbytes of sb to `to` while receiving rbytes into rb from `from` (either side may be empty)
    virtual int shift(int to, const char *sb, size_t sbytes, int from, char *rb, size_t rbytes) = 0;
    int xchg(int peer, const char *sb, size_t sbytes, char *rb, size_t rbytes) {
        return shift(peer, sb, sbytes, peer, rb, rbytes);
    }
};
// redscat: the pre-step of MPIR_Reduce_redscat_gather_MV2 (reduce_osu.c:849-894) instead — the odd
// ranks below 2 * rem hand their operand to rank - 1 — with the allgather standing for its gather
// to the root and the broadcast after it (MPI_Iallreduce's naive schedule moves the blocks only).
int sched_allreduce(Xport &x, int n, int rank, char *acc, char *tmp, size_t count, size_t ext, int dtype, int op,
                    bool rd, bool redscat = false) {
    int pof2 = 1;
    while (pof2 * 2 <= n) pof2 *= 2;
    const int rem = n - pof2;
    const size_t S = count * ext;
    int rc = 0, newrank;
    auto uop = [&](size_t off, size_t cnt) { return mv2h_reduce_local(tmp + off, acc + off, cnt, dtype, op, nullptr); };
    // non-power-of-two pre-step: even ranks below 2 * rem hand their operand to rank + 1 (redscat:
    // the odd ones to rank - 1)
    const int hand = redscat ? 1 : 0, keep = 1 - hand;
    if (rank < 2 * rem) {
        if (rank % 2 == hand) {
            if ((rc = x.xchg(hand ? rank - 1 : rank + 1, acc, S, nullptr, 0))) return rc;
            newrank = -1;
        } else {
            if ((rc = x.xchg(hand ? rank + 1 : rank - 1, nullptr, 0, tmp, S)) || (rc = uop(0, count))) return rc;
            newrank = rank / 2;
        }
    } else {
        newrank = rank - rem;
    }
    auto real = [&](int nr) { return nr < rem ? nr * 2 + keep : nr + rem; };
    if (newrank != -1 && (rd || count < (size_t)pof2)) {
        for (int mask = 1; mask < pof2; mask <<= 1) {
            if ((rc = x.xchg(real(newrank ^ mask), acc, S, tmp, S)) || (rc = uop(0, count))) return rc;
        }
    } else if (newrank != -1) {
        // reduce-scatter by recursive halving over pof2 blocks (the last one takes the remainder),
        // then the recursive-doubling allgather
        std::vector<size_t> cnts((size_t)pof2, count / (size_t)pof2), disps((size_t)pof2, 0);
        cnts[(size_t)pof2 - 1] = count - (count / (size_t)pof2) * (size_t)(pof2 - 1);
        for (int i = 1; i < pof2; ++i) disps[i] = disps[i - 1] + cnts[i - 1];
        auto span = [&](int a, int b) { return a < b ? disps[b - 1] + cnts[b - 1] - disps[a] : (size_t)0; };
        int mask = 1, send_idx = 0, recv_idx = 0, last_idx = pof2;
        while (mask < pof2) {
            const int newdst = newrank ^ mask;
            size_t scnt, rcnt;
            if (newrank < newdst) {
                send_idx = recv_idx + pof2 / (mask * 2);
                scnt = span(send_idx, last_idx);
                rcnt = span(recv_idx, send_idx);
            } else {
                recv_idx = send_idx + pof2 / (mask * 2);
                scnt = span(send_idx, recv_idx);
                rcnt = span(recv_idx, last_idx);
            }
            const size_t so = disps[send_idx] * ext, ro = disps[recv_idx] * ext;
            if ((rc = x.xchg(real(newdst), acc + so, scnt * ext, tmp + ro, rcnt * ext)) || (rc = uop(ro, rcnt)))
                return rc;
            send_idx = recv_idx;
            mask <<= 1;
            if (mask < pof2) last_idx = recv_idx + pof2 / mask;
        }
        for (mask >>= 1; mask > 0; mask >>= 1) {
            const int newdst = newrank ^ mask;
            size_t scnt, rcnt;
            if (newrank < newdst) {
                if (mask != pof2 / 2) last_idx = last_idx + pof2 / (mask * 2);
                recv_idx = send_idx + pof2 / (mask * 2);
                scnt = span(send_idx, recv_idx);
                rcnt = span(recv_idx, last_idx);
            } else {
                recv_idx = send_idx - pof2 / (mask * 2);
                scnt = span(send_idx, last_idx);
                rcnt = span(recv_idx, send_idx);
            }
            if ((rc = x.xchg(real(newdst), acc + disps[send_idx] * ext, scnt * ext, acc + disps[recv_idx] * ext,
                             rcnt * ext)))
                return rc;
            if (newrank > newdst) send_idx = recv_idx;
        }
    }
    // post-step: the ranks that kept their place below 2 * rem return the result to the others
    if (rank < 2 * rem) {
        const int peer = rank % 2 ? rank - 1 : rank + 1;
        rc = rank % 2 == keep ? x.xchg(peer, acc, S, nullptr, 0) : x.xchg(peer, nullptr, 0, acc, S);
    }
    return rc;
}

// MPIR_Reduce_binomial_MV2's commutative schedule (reduce_osu.c:577-663; MPIR_Ireduce_binomial
// reduces the same way): relative rank rel receives from rel | mask and reduces uop(tmp, acc)
// until its bit `mask` is set, then sends its partial to rel & ~mask.  acc ends with the result
// at the root.
int sched_binomial_reduce(Xport &x, int n, int rank, int root, char *acc, char *tmp, size_t count, size_t ext,
                          int dtype, int op) {
    const int rel = (rank - root + n) % n;
    const size_t S = count * ext;
    int rc = 0;
    for (int mask = 1; mask < n; mask <<= 1) {
        if (rel & mask) return x.xchg(((rel & ~mask) + root) % n, acc, S, nullptr, 0);
        if ((rel | mask) < n && ((rc = x.xchg(((rel | mask) + root) % n, nullptr, 0, tmp, S)) ||
                                 (rc = mv2h_reduce_local(tmp, acc, count, dtype, op, nullptr))))
            return rc;
    }
    return 0;
}

// MPIR_Reduce_knomial_MV2 (reduce_osu.c:1639-1837) as messages: the children of
// MPIR_Reduce_knomial_trace (:1568-1633: k - 1 per mask, masks from the largest down) send their
// partials; the receives are posted from the trace's last child to its first (:1735-1741) and
// reduced uop(tmp, acc) in request-index order (the Waitany order restated), then the
// partial goes to the parent.  acc ends with the result at the root (commutative ops only, as in
// the reference's dispatch, :2637-2644).
int sched_knomial_reduce(Xport &x, int n, int rank, int root, int k, char *acc, char *tmp, size_t count, size_t ext,
                         int dtype, int op) {
    const int rel = (rank - root + n) % n;
    const size_t S = count * ext;
    int mask = 1, dst = -1;
    while (mask < n) {
        if (rel % (k * mask)) {
            dst = rel / (k * mask) * (k * mask) + root;
            if (dst >= n) dst -= n;
            break;
        }
        mask *= k;
    }
    mask /= k;
    std::vector<int> src;
    for (int m = mask; m > 0; m /= k)
        for (int j = 1; j < k; ++j)
            if (rel + m * j < n) src.push_back(rank + m * j >= n ? rank + m * j - n : rank + m * j);
    int rc = 0;
    for (size_t i = src.size(); i-- > 0;)
        if ((rc = x.xchg(src[i], nullptr, 0, tmp, S)) || (rc = mv2h_reduce_local(tmp, acc, count, dtype, op, nullptr)))
            return rc;
    return dst >= 0 ? x.xchg(dst, acc, S, nullptr, 0) : 0;
}

// the node leaders as ranks (node index), over their TCP links, staged through g_mn.h0 / h1
struct LeaderLinks : Xport {
    int shift(int to, const char *sb, size_t sbytes, int from, char *rb, size_t rbytes) override {
        int rc = 0;
        if (sbytes && (rc = mn_d2h(g_mn.h0, sb, sbytes))) return rc;
        if (sbytes && rbytes) rc = net_shift(to, g_mn.h0, sbytes, from, g_mn.h1, rbytes);
        else if (sbytes) rc = net_send(to, g_mn.h0, sbytes);
        else if (rbytes) rc = net_recv(from, g_mn.h1, rbytes);
        return rc || !rbytes ? rc : mn_h2d(rb, g_mn.h1, rbytes);
    }
};

// every rank of the job (global rank), over the point-to-point channels in the library's
// collective context: device IPC within a node, the rank mesh between nodes
struct RankChannels : Xport {
    int shift(int to, const char *sb, size_t sbytes, int from, char *rb, size_t rbytes) override {
        unsigned long long sq = 0, rq = 0;
        int rc = 0;
        if (rbytes && (rc = p2p_irecv(rb, rbytes, from, kCollTagBase - 3, &rq))) return rc;
        if (sbytes && (rc = p2p_isend(sb, sbytes, to, kCollTagBase - 3, &sq))) {
            if (rq) p2p_abandon(rq);  // withdrawn, or the context poisoned: never matched into later
            return rc;
        }
        if (sbytes && (rc = mv2h_p2p_wait(sq, nullptr, nullptr, nullptr))) {
            p2p_abandon(sq);
            if (rq) p2p_abandon(rq);
            return rc;
        }
        if (rbytes && (rc = mv2h_p2p_wait(rq, nullptr, nullptr, nullptr))) p2p_abandon(rq);
        return rc;
    }
};

// MPI_Reduce_scatter's message schedules over n ranks (commutative ops, every uop one device
// Reduce_local of the received data `in` into this rank's accumulator `inout`).  in: this rank's
// whole operand (device, total elements, block j at disps[j]); out: its block (cnts[rank]
// elements, device or host); t0 / t1: device scratch of the whole operand.
//
// MPIR_Reduce_scatter_Rec_Halving_MV2 (red_scat_osu.c:428-780): the non-power-of-two pre-step,
// recursive halving over pof2 merged blocks (an odd rank below 2 * rem also works its left
// neighbour's block), the post-step returning the even ranks' blocks.
int sched_rs_halving(Xport &x, int n, int rank, const size_t *cnts, const size_t *disps, const char *in, char *out,
                     char *t0, char *t1, size_t ext, int dtype, int op) {
    const size_t total = disps[n - 1] + cnts[n - 1], S = total * ext;
    char *res = t0, *tmp = t1;  // tmp_results, tmp_recvbuf
    if (hipMemcpy(res, in, S, hipMemcpyDefault) != hipSuccess) return E_INTERN;
    int pof2 = 1;
    while (pof2 * 2 <= n) pof2 *= 2;
    const int rem = n - pof2;
    int rc = 0, newrank;
    if (rank < 2 * rem) {
        if (rank % 2 == 0) {
            if ((rc = x.xchg(rank + 1, res, S, nullptr, 0))) return rc;
            newrank = -1;
        } else {
            if ((rc = x.xchg(rank - 1, nullptr, 0, tmp, S)) ||
                (rc = mv2h_reduce_local(tmp, res, total, dtype, op, nullptr)))
                return rc;
            newrank = rank / 2;
        }
    } else {
        newrank = rank - rem;
    }
    auto real = [&](int nr) { return nr < rem ? nr * 2 + 1 : nr + rem; };
    if (newrank != -1) {
        std::vector<size_t> ncnt((size_t)pof2), ndisp((size_t)pof2, 0);
        for (int i = 0; i < pof2; ++i) {
            const int old = real(i);
            ncnt[i] = cnts[old] + (old < 2 * rem ? cnts[old - 1] : 0);
        }
        for (int i = 1; i < pof2; ++i) ndisp[i] = ndisp[i - 1] + ncnt[i - 1];
        auto span = [&](int a, int b) {
            size_t c = 0;
            for (int i = a; i < b; ++i) c += ncnt[i];
            return c;
        };
        int send_idx = 0, recv_idx = 0, last_idx = pof2;
        for (int mask = pof2 >> 1; mask > 0; mask >>= 1) {
            const int newdst = newrank ^ mask;
            size_t scnt, rcnt;
            if (newrank < newdst) {
                send_idx = recv_idx + mask;
                scnt = span(send_idx, last_idx);
                rcnt = span(recv_idx, send_idx);
            } else {
                recv_idx = send_idx + mask;
                scnt = span(send_idx, recv_idx);
                rcnt = span(recv_idx, last_idx);
            }
            const size_t so = ndisp[send_idx] * ext, ro = ndisp[recv_idx] * ext;
            if ((rc = x.xchg(real(newdst), res + so, scnt * ext, tmp + ro, rcnt * ext))) return rc;
            if (rcnt && (rc = mv2h_reduce_local(tmp + ro, res + ro, rcnt, dtype, op, nullptr))) return rc;
            send_idx = recv_idx;
            last_idx = recv_idx + mask;
        }
        if (cnts[rank] &&
            hipMemcpy(out, res + disps[rank] * ext, cnts[rank] * ext, hipMemcpyDefault) != hipSuccess)
            return E_INTERN;
    }
    if (rank < 2 * rem) {
        if (rank % 2) rc = x.xchg(rank - 1, res + disps[rank - 1] * ext, cnts[rank - 1] * ext, nullptr, 0);
        else if (is_device(out)) rc = x.xchg(rank + 1, nullptr, 0, out, cnts[rank] * ext);
        else if (!(rc = x.xchg(rank + 1, nullptr, 0, tmp, cnts[rank] * ext)) && cnts[rank])
            rc = hipMemcpy(out, tmp, cnts[rank] * ext, hipMemcpyDefault) == hipSuccess ? 0 : E_INTERN;
    }
    return rc;
}

// MPIR_Reduce_scatter_Pair_Wise_MV2 (:786-1020): this rank's block starts as its own data; step i
// sends block (rank + i) to that rank and reduces the block received from rank - i into it
int sched_rs_pairwise(Xport &x, int n, int rank, const size_t *cnts, const size_t *disps, const char *in, char *out,
                      char *t0, char *t1, size_t ext, int dtype, int op) {
    const size_t B = cnts[rank] * ext;
    if (B && hipMemcpy(t0, in + disps[rank] * ext, B, hipMemcpyDefault) != hipSuccess) return E_INTERN;
    int rc = 0;
    for (int i = 1; i < n; ++i) {
        const int src = (rank - i + n) % n, dst = (rank + i) % n;
        if ((rc = x.shift(dst, in + disps[dst] * ext, cnts[dst] * ext, src, t1, B))) return rc;
        if (B && (rc = mv2h_reduce_local(t1, t0, cnts[rank], dtype, op, nullptr))) return rc;
    }
    return !B || hipMemcpy(out, t0, B, hipMemcpyDefault) == hipSuccess ? 0 : E_INTERN;
}

// MPIR_Reduce_scatter_ring(_2lvl) (:1026-1180, :1190-1300; its 1 MiB chunking does not change an
// element's order): at distance d this rank sends block (rank + d) to the right, having reduced the
// partial received from the left into its own data of that block
int sched_rs_ring(Xport &x, int n, int rank, const size_t *cnts, const size_t *disps, const char *in, char *out,
                  char *t0, char *t1, size_t ext, int dtype, int op) {
    const int right = (rank + 1) % n, left = (rank - 1 + n) % n;
    int rc = 0;
    for (int dist = n - 1; dist >= 0; --dist) {
        const int sr = (rank + dist) % n, rr = (rank + dist - 1 + n) % n;
        const size_t sc = cnts[sr];
        if (sc && hipMemcpy(t0, in + disps[sr] * ext, sc * ext, hipMemcpyDefault) != hipSuccess) return E_INTERN;
        if (dist < n - 1 && sc && (rc = mv2h_reduce_local(t1, t0, sc, dtype, op, nullptr))) return rc;
        if (dist > 0) {
            if ((rc = x.shift(right, t0, sc * ext, left, t1, cnts[rr] * ext))) return rc;
        } else if (sc && hipMemcpy(out, t0, sc * ext, hipMemcpyDefault) != hipSuccess) {
            return E_INTERN;
        }
    }
    return 0;
}

// leaders: recursive doubling on `acc` (device, `count` elements) with the nodes as ranks
int leader_rd(char *acc, size_t count, int dtype, int op, size_t bytes) {
    World &w = world();
    LeaderLinks x;
    return sched_allreduce(x, w.nnodes, w.node, acc, g_mn.d1, count, bytes / count, dtype, op, true);
}

// leaders: binomial broadcast of the host buffer h from node `root` (MPIR_Bcast_binomial order)
int leader_bcast(char *h, size_t bytes, int root) {
    World &w = world();
    const int n = w.nnodes, rel = (w.node - root + n) % n;
    int mask = 1, rc = 0;
    while (mask < n) {
        if (rel & mask) {
            if ((rc = net_recv((w.node - mask + n) % n, h, bytes))) return rc;
            break;
        }
        mask <<= 1;
    }
    for (mask >>= 1; mask > 0; mask >>= 1)
        if (rel + mask < n && (rc = net_send((w.node + mask) % n, h, bytes))) return rc;
    return 0;
}
}  // namespace

static int mn_require_device_reduction(int dtype, int op) {
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc) return rc;
    return kind_supported(dt);
}

// MPIR_Allreduce_index_tuned_intra_MV2's selection (allreduce_osu.c:3015-3373) over the whole job.
// Returns 0 (two-level), 1 (flat ring wrapper), or ALG_PT2PT_RS / ALG_PT2PT_RD (flat over every
// rank).  The small-message shortcuts (:118-160) keep the two-level structure; the skip-large gate
// (:163-171) takes the ring wrapper; then the tuning tables (orders.cpp mn_allreduce_table).
static int mn_select(int ppn, int gsize, long nbytes, int *intra, int *inter) {
    const Knobs &K = knobs();
    *intra = MN_INTRA_NODE;  // the shortcuts' node step is the node's own small-message order
    *inter = ALG_PT2PT_RD;   // and their leaders' step recursive doubling (:2215-2262, :147-153)
    bool tables = false;
    if (K.allred_skip_small) {
        if (nbytes <= K.topo_allred_max && nbytes >= K.topo_allred_min && K.enable_topo && K.use_topo_allreduce) {
            if (ppn >= K.topo_allred_ppn) return 0;  // topology-aware hierarchical
            tables = true;                           // goto use_tables
        }
        if (!tables && K.enable_shmem_allreduce && K.enable_skip_search && nbytes <= K.coll_skip_thr) return 0;
    }
    if (!tables && K.allred_skip_large && K.allred_use_ring == 1 && K.allred_ring_thr <= nbytes &&
        ppn <= K.allred_ring_ppn)
        return 1;
    int in = MN_INTRA_NODE, it = ALG_PT2PT_RD;
    const int t = mn_allreduce_table(ppn, gsize, nbytes, &in, &it);
    if (t == 0) {
        *intra = in;
        *inter = it;
        return 0;
    }
    return t;
}

// How a multi-node call with a builtin op runs (a pure function of the job's shape and the call,
// so every rank takes the same route; mv2h_mn_route exposes it to the CPU tests).  A flat
// algorithm runs as per-element programs up to kMaxRanks ranks (MN_FLAT_PROG), as its message
// schedule over the rank channels up to kMeshMaxRanks (MN_SCHED: the rank mesh exists up to
// there), and above that the two-level structure stands in for it (MN_FALLBACK: Allreduce and
// Iallreduce the two-level allreduce with the default node and leader steps, Ireduce the
// two-level reduce helper, Reduce_scatter the basic algorithm) — correct for every builtin op,
// its fp order not the reference's (unpinned; integer, bitwise, logical and LOC results exact).
enum MnRoute { MN_TWO_LEVEL_R = 0, MN_RING_R = 1, MN_FLAT_PROG = 2, MN_SCHED = 3, MN_FALLBACK = 4, MN_BASIC_R = 5 };
static int mn_flat_route(int gsize) {
    return gsize <= mn_prog_max() ? MN_FLAT_PROG : gsize <= kMeshMaxRanks ? MN_SCHED : MN_FALLBACK;
}
// MPI_Allreduce / MPI_Iallreduce (nbc = the call's mv2h_nbc kind).  *rem_route: the route of the
// ring wrapper's count % gsize remainder (pt2pt_rs over every rank), -1 when there is none.
static int mn_allreduce_route(int ppn, int gsize, long nbytes, size_t count, bool in_place, int nbc, int *intra,
                              int *inter, int *sel_out, int *rem_route) {
    *intra = MN_INTRA_NODE;
    *inter = ALG_PT2PT_RD;
    *sel_out = 0;
    *rem_route = -1;
    if (nbc == NBC_IALLREDUCE) return mn_flat_route(gsize);
    const int sel = mn_select(ppn, gsize, nbytes, intra, inter);
    *sel_out = sel;
    if (sel == 1) {
        if (!in_place && count >= (size_t)gsize) {
            if (count % (size_t)gsize) *rem_route = mn_flat_route(gsize);
            return MN_RING_R;
        }
        return mn_flat_route(gsize);
    }
    if (sel == ALG_PT2PT_RS || sel == ALG_PT2PT_RD) return mn_flat_route(gsize);
    return MN_TWO_LEVEL_R;
}
// MPI_Reduce_scatter / MPI_Ireduce_scatter over gsize ranks, nbytes in all
static int mn_reduce_scatter_route(int gsize, long nbytes) {
    if (reduce_scatter_algo(gsize, nbytes) == ALG_RS_BASIC) return MN_BASIC_R;
    const int r = mn_flat_route(gsize);
    return r == MN_FALLBACK ? MN_BASIC_R : r;
}
// MPIR_Reduce_index_tuned_intra_MV2 across nodes (reduce_osu.c:2498-2660) for a commutative op
// (opk: builtin or commutative user op; a non-commutative one always takes the flat binomial,
// :2628-2636): two_level = MPIR_Reduce_two_level_helper_MV2 with the node step `intra` to local rank
// 0 and `algo` over the leaders to the root's node; else `algo` flat over every rank.  The
// small-message shortcut (:2508-2514: up to MV2_COLL_SKIP_TABLE_THRESHOLD, shmem + binomial) and the
// tables (orders.cpp mn_reduce_table).  The helper's MPIR_Reduce_shmem_MV2 node step becomes the intra
// knomial wrapper from the shmem slot size on (:2240-2251); the flat knomial needs a commutative op and
// the flat redscat_gather a builtin op with count >= pof2 (:2637-2652), else binomial.  The
// topology-aware reduce (:2498-2506, off by default) is not restated across nodes.
struct MnRedSel {
    bool two_level;
    int intra, algo, k;
};
static int floor_pof2(int n) {
    int p = 1;
    while (p * 2 <= n) p *= 2;
    return p;
}
static MnRedSel mn_reduce_select(int ppn, int gsize, size_t count, int tsize, int textent, int opk) {
    const Knobs &K = knobs();
    const long nbytes = (long)count * tsize;
    MnReduceCell c{};
    MnRedSel r{true, ALG_SHMEM_LINEAR, ALG_BINOMIAL, 4};
    if (opk == OPK_USER_NONCOMM) return MnRedSel{false, 0, ALG_BINOMIAL, 4};
    if (!(K.enable_shmem_reduce && K.enable_skip_search && nbytes <= K.coll_skip_thr)) {
        mn_reduce_table(ppn, gsize, nbytes, &c);
        r = MnRedSel{c.two_level != 0, c.intra, c.inter, c.k};
    } else {
        mn_reduce_table(ppn, gsize, nbytes, &c);  // the knomial factor only
        r.k = c.k;
    }
    if (r.two_level) {
        if (r.intra == ALG_SHMEM_LINEAR && !(K.enable_shmem_reduce && (long)count * textent < K.shmem_coll_max_msg))
            r.intra = ALG_KNOMIAL;
        return r;
    }
    if (r.algo == ALG_REDSCAT_GATHER && !(opk == OPK_BUILTIN && count >= (size_t)floor_pof2(gsize))) r.algo = ALG_BINOMIAL;
    return r;
}
// MPI_Reduce / MPI_Ireduce: MN_TWO_LEVEL_R (the helper), or a flat algorithm's route
static int mn_reduce_route(int ppn, int gsize, size_t count, int tsize, int nbc) {
    if (nbc == NBC_IREDUCE) return mn_flat_route(gsize);
    const MnRedSel sel = mn_reduce_select(ppn, gsize, count, tsize, tsize, OPK_BUILTIN);
    return sel.two_level ? MN_TWO_LEVEL_R : mn_flat_route(gsize);
}

static int mn_allreduce_2lvl(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream,
                             int intra = MN_INTRA_NODE, int inter = ALG_PT2PT_RD);
static int mn_flat_allreduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream,
                             int algo, int root = -1, const Plan *forced = nullptr);

// The node's S-byte operands at its leader only (G: L * S bytes, local rank order; unused on the
// other ranks), over the node's device point-to-point channels in the library's collective context
static int gather_node_leader(const void *mine, char *G, size_t S) {
    World &w = world();
    const int L = w.size, base = w.node * w.size;  // point-to-point takes global ranks
    unsigned long long req[kMaxRanks] = {};
    int rc = 0;
    if (w.rank != 0) {
        if ((rc = p2p_isend(mine, S, base, kCollTagBase - 2, &req[0]))) return rc;
        return mv2h_p2p_wait(req[0], nullptr, nullptr, nullptr);
    }
    for (int l = 1; l < L; ++l)
        if ((rc = p2p_irecv(G + (size_t)l * S, S, base + l, kCollTagBase - 2, &req[l]))) return rc;
    if (hipMemcpy(G, mine, S, hipMemcpyDefault) != hipSuccess) return E_INTERN;
    for (int l = 1; l < L; ++l)
        if ((rc = mv2h_p2p_wait(req[l], nullptr, nullptr, nullptr))) return rc;
    return 0;
}

// Flat ring over every rank of the job (MPIR_Allreduce_pt2pt_ring_MV2, allreduce_osu.c:3916-3968):
// chunk c of (count / n) elements ends as x_c (+) x_{c+1} (+) ... (+) x_{c-1} over the global ranks,
// the accumulator always inout (uop(comp_chunk, recv_chunk), :3958).  Here each node gathers its
// ranks' operands, and the node leaders pass partial chunks round the ring of nodes: group g (the
// chunks of node g's ranks) starts at node g with the ranks from the chunk's own onwards, crosses
// every other node whole, and ends at node g with the ranks before it.  Every uop is one device
// Reduce_local.  The wrapper's remainder (count % n elements, pt2pt_rs over every rank, :3800-3818)
// is that flat algorithm (its programs up to kMaxRanks ranks, its message schedule above).
static int mn_ring_allreduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream) {
    World &w = world();
    const DtypeInfo *dt = dtype_lookup(dtype);
    const size_t ext = (size_t)dt->extent, S = count * ext;
    const int L = w.size, K = w.nnodes, n = w.gsize;
    const size_t cc = count / (size_t)n, cb = cc * ext, sect = (size_t)L * cb, main_bytes = (size_t)K * sect;
    const int chain[3] = {PV_AR_RING_WRAPPER, PV_AR_RING, PV_AR_SHM_RS};
    pvar_note_ids(chain, count % (size_t)n ? 3 : 2);
    int rc = 0;
    if (w.rank == 0) {
        char *G = (char *)get_scratch(6, (size_t)L * S);  // the node's operands, local rank order
        if (!G) return E_NO_MEM;
        if ((rc = gather_node_leader(sendbuf, G, S))) return rc;
        if ((rc = mn_reserve(std::max(main_bytes, sect)))) return rc;
        char *A = g_mn.d0;  // partial chunks of the group in hand
        auto X = [&](int l, size_t byte_off) { return (const char *)G + (size_t)l * S + byte_off; };
        const int me = w.node, right = (me + 1) % K, left = (me - 1 + K) % K;
        // round 0: this node's group, from each chunk's own rank to the node's last
        for (int l = 0; l < L; ++l) {
            const size_t off = ((size_t)me * L + l) * cb;
            if (hipMemcpy(A + (size_t)l * cb, X(l, off), cb, hipMemcpyDeviceToDevice) != hipSuccess) return E_INTERN;
            for (int m = l + 1; m < L; ++m)
                if ((rc = mv2h_reduce_local(X(m, off), A + (size_t)l * cb, cc, dtype, op, nullptr))) return rc;
        }
        for (int t = 1; t <= K; ++t) {
            if ((rc = mn_d2h(g_mn.h0, A, sect)) || (rc = net_shift(right, g_mn.h0, sect, left, g_mn.h1, sect)) ||
                (rc = mn_h2d(A, g_mn.h1, sect)))
                return rc;
            const int g = (me - t + K) % K;
            if (t < K) {  // a whole node: its ranks in order, all of the group's chunks at once
                for (int m = 0; m < L; ++m)
                    if ((rc = mv2h_reduce_local(X(m, (size_t)g * sect), A, cc * (size_t)L, dtype, op, nullptr)))
                        return rc;
            } else {  // back home: the ranks before each chunk's own
                for (int l = 0; l < L; ++l)
                    for (int m = 0; m < l; ++m)
                        if ((rc = mv2h_reduce_local(X(m, ((size_t)me * L + l) * cb), A + (size_t)l * cb, cc, dtype,
                                                    op, nullptr)))
                            return rc;
            }
        }
        // allgather of the groups over the leaders (data movement only), then into recvbuf
        if ((rc = mn_d2h(g_mn.h1 + (size_t)me * sect, A, sect))) return rc;
        for (int k = 0; k < K - 1; ++k) {
            const int so = (me - k + K) % K, ro = (me - k - 1 + K) % K;
            if ((rc = net_shift(right, g_mn.h1 + (size_t)so * sect, sect, left, g_mn.h1 + (size_t)ro * sect, sect)))
                return rc;
        }
        if ((rc = mn_h2d(recvbuf, g_mn.h1, main_bytes))) return rc;
    } else if ((rc = gather_node_leader(sendbuf, nullptr, S))) {
        return rc;
    }
    if ((rc = bcast_node(recvbuf, main_bytes, 0, stream))) return rc;
    if (count % (size_t)n == 0) return 0;
    // the wrapper's pt2pt_rs over every rank (recursive doubling: rem < n)
    return mn_flat_allreduce((const char *)sendbuf + main_bytes, (char *)recvbuf + main_bytes, count % (size_t)n,
                             dtype, op, stream, ALG_PT2PT_RS);
}

// Every rank's S-byte operand onto every rank, in global rank order (*out: device scratch of
// gsize * S bytes): node allgather into the node's section, a ring of sections over the leaders,
// node broadcast.  The data movement of the flat algorithms restated across nodes.
static int mn_gather_all(const void *mine, size_t S, char **out, void *stream) {
    World &w = world();
    const int n = w.gsize, K = w.nnodes;
    const size_t sect = (size_t)w.size * S;
    char *W = (char *)get_scratch(6, (size_t)n * S);
    if (!W) return E_NO_MEM;
    int rc = 0;
    if (w.rank == 0 && (rc = mn_reserve_host((size_t)n * S))) return rc;
    if ((rc = allgather_node(mine, W + (size_t)w.node * sect, S, stream))) return rc;
    if (w.rank == 0) {
        const int me = w.node, right = (me + 1) % K, left = (me - 1 + K) % K;
        if ((rc = mn_d2h(g_mn.h0 + (size_t)me * sect, W + (size_t)me * sect, sect))) return rc;
        for (int k = 0; k < K - 1; ++k) {
            const int so = (me - k + K) % K, ro = (me - k - 1 + K) % K;
            if ((rc = net_shift(right, g_mn.h0 + (size_t)so * sect, sect, left, g_mn.h0 + (size_t)ro * sect, sect)))
                return rc;
        }
        if ((rc = mn_h2d(W, g_mn.h0, (size_t)n * S))) return rc;
    }
    if ((rc = bcast_node(W, (size_t)n * S, 0, stream))) return rc;
    *out = W;
    return 0;
}

// Flat pt2pt_rs / pt2pt_rd over more than kMaxRanks ranks (beyond the programs' registers): the
// algorithm's message schedule itself (sched_allreduce) over every rank's point-to-point channels,
// each step's received data reduced into this rank's accumulator (recvbuf, or device scratch when
// recvbuf is host memory) by one device Reduce_local.
static int mn_sched_allreduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, int algo) {
    World &w = world();
    const DtypeInfo *dt = dtype_lookup(dtype);
    const bool in_place = sendbuf == (const void *)-1;
    const size_t ext = (size_t)dt->extent, S = count * ext;
    if (w.gsize > kMeshMaxRanks) return E_UNSUPPORTED;  // no rank mesh: every rank refuses alike
    const int id = algo == ALG_PT2PT_RS ? PV_AR_SHM_RS : PV_AR_SHM_RD;
    pvar_note_ids(&id, 1);
    int rc = mn_reserve_dev(S);
    if (rc) return rc;
    char *acc = is_device(recvbuf) ? (char *)recvbuf : g_mn.d0;
    const void *src = in_place ? recvbuf : sendbuf;
    if (src != acc && hipMemcpy(acc, src, S, hipMemcpyDefault) != hipSuccess) return E_INTERN;
    RankChannels x;
    if ((rc = sched_allreduce(x, w.gsize, w.grank, acc, g_mn.d1, count, ext, dtype, op, algo == ALG_PT2PT_RD)))
        return rc;
    return acc == recvbuf || hipMemcpy(recvbuf, acc, S, hipMemcpyDefault) == hipSuccess ? 0 : E_INTERN;
}

// MVAPICH2's nonblocking schedules over more than kMaxRanks ranks, as messages: root >= 0
// MPI_Ireduce = MPIR_Ireduce_binomial to the root (ireduce_osu.c -> ireduce_tuning.c first row);
// root < 0 MPI_Iallreduce = MPIR_Iallreduce_naive (iallreduce.c:109-139): MPIR_Ireduce_intra to
// rank 0 — redscat_gather for builtin ops above MPIR_CVAR_REDUCE_SHORT_MSG_SIZE with count >= pof2
// (ireduce.c:700-731), else binomial — then MPIR_Ibcast, every rank taking rank 0's result.
static int mn_bcast(void *buffer, size_t bytes, int root, void *stream);
static int mn_sched_naive(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream,
                          int root) {
    World &w = world();
    const DtypeInfo *dt = dtype_lookup(dtype);
    const bool in_place = sendbuf == (const void *)-1;
    const size_t ext = (size_t)dt->extent, S = count * ext;
    const int n = w.gsize, me = w.grank;
    if (n > kMeshMaxRanks) return E_UNSUPPORTED;  // no rank mesh: every rank refuses alike
    int rc = mn_reserve_dev(S);
    if (rc) return rc;
    // the accumulator: recvbuf where it is significant and device memory, else device scratch
    const bool mine = (root < 0 || me == root) && recvbuf && is_device(recvbuf);
    char *acc = mine ? (char *)recvbuf : g_mn.d0;
    const void *src = in_place ? recvbuf : sendbuf;
    if (src != acc && hipMemcpy(acc, src, S, hipMemcpyDefault) != hipSuccess) return E_INTERN;
    RankChannels x;
    int pof2 = 1;
    while (pof2 * 2 <= n) pof2 *= 2;
    if (root < 0 && (long)(count * (size_t)dt->size) > knobs().reduce_short_msg && count >= (size_t)pof2) {
        rc = sched_allreduce(x, n, me, acc, g_mn.d1, count, ext, dtype, op, false, true);
    } else {
        rc = sched_binomial_reduce(x, n, me, root < 0 ? 0 : root, acc, g_mn.d1, count, ext, dtype, op);
        if (!rc && root < 0) rc = mn_bcast(acc, S, 0, stream);
    }
    if (rc || (root >= 0 && me != root) || acc == recvbuf) return rc;
    return hipMemcpy(recvbuf, acc, S, hipMemcpyDefault) == hipSuccess ? 0 : E_INTERN;
}

// Flat pt2pt_rs / pt2pt_rd over every rank (allreduce_osu.c:633-1054, :360-630): every rank's operand reaches every rank
// (node allgather into its global slot, a ring over the leaders, node broadcast), and each rank
// evaluates the algorithm's per-element programs for its own rank — recursive doubling's results
// differ between ranks where the op is not commutative in its bits (MAX/MIN ties of ±0, NaN
// payloads), as the reference's do.  algo 0: the plan of the call's own selection (a nonblocking
// call's: MPIR_Iallreduce_naive = Ireduce to rank 0 + Ibcast, every rank takes rank 0's result).
// root >= 0 (MPI_Ireduce): only the root evaluates, the plan of MPIR_Ireduce_binomial.
static int mn_flat_allreduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream,
                             int algo, int root, const Plan *forced) {
    World &w = world();
    const DtypeInfo *dt = dtype_lookup(dtype);
    const bool in_place = sendbuf == (const void *)-1;
    const size_t S = count * (size_t)dt->extent;
    const int n = w.gsize;
    if (n > mn_prog_max() && root < 0 && (algo == ALG_PT2PT_RS || algo == ALG_PT2PT_RD))
        return mn_flat_route(n) == MN_SCHED ? mn_sched_allreduce(sendbuf, recvbuf, count, dtype, op, algo)
                                            : mn_allreduce_2lvl(sendbuf, recvbuf, count, dtype, op, stream);
    Plan p;
    int rc = forced ? (p = *forced, 0)
             : root >= 0 ? plan_reduce(n, w.grank, root, count, dt->size, dt->extent, &p)
                         : plan_allreduce(n, w.grank, count, dt->size, dt->extent, in_place, algo, &p);
    if (rc) return rc;
    pvar_note(root >= 0 ? PV_COLL_REDUCE : PV_COLL_ALLREDUCE, p, in_place, count, n);
    char *W = nullptr;  // every rank's operand, global rank order
    if ((rc = mn_reserve_dev(S)) || (rc = mn_gather_all(in_place ? recvbuf : sendbuf, S, &W, stream))) return rc;
    if (root >= 0 && w.grank != root) return 0;
    const void *srcs[kMaxRanks];
    for (int r = 0; r < n; ++r) srcs[r] = W + (size_t)r * S;
    if ((rc = mv2h_reduce_n_prog(srcs, n, g_mn.d1, count, dtype, op, (const mv2h_progset *)&p.ps, nullptr)))
        return rc;
    return hipMemcpy(recvbuf, g_mn.d1, S, hipMemcpyDefault) == hipSuccess ? 0 : E_INTERN;
}

static int mn_allreduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream) {
    int rc = mn_require_device_reduction(dtype, op);
    if (rc || count == 0) return rc;
    const World &w = world();
    const DtypeInfo *dt = dtype_lookup(dtype);
    const bool in_place = sendbuf == (const void *)-1;
    const int gsize = w.gsize;
    int intra = MN_INTRA_NODE, inter = ALG_PT2PT_RD, sel = 0, rem = -1;
    const int route = mn_allreduce_route(w.size, gsize, (long)(count * (size_t)dt->size), count, in_place, nbc_kind(),
                                         &intra, &inter, &sel, &rem);
    // MPI_Iallreduce: MVAPICH2's nonblocking schedule is flat over the whole job
    // (MPIR_Iallreduce_intra_MV2 iallreduce_osu.c:257 -> MPIR_Iallreduce_naive: Ireduce to rank 0,
    // binomial or redscat_gather, then Ibcast), whatever the nodes
    if (nbc_kind() == NBC_IALLREDUCE) {
        if (route == MN_FLAT_PROG) return mn_flat_allreduce(sendbuf, recvbuf, count, dtype, op, stream, 0);
        if (route == MN_SCHED) return mn_sched_naive(sendbuf, recvbuf, count, dtype, op, stream, -1);
        return mn_allreduce_2lvl(sendbuf, recvbuf, count, dtype, op, stream);
    }
    if (route == MN_RING_R) return mn_ring_allreduce(sendbuf, recvbuf, count, dtype, op, stream);
    if (sel == 1) {
        // the wrapper's ring body needs count >= n and a separate sendbuf (:3893-3898); otherwise
        // it runs pt2pt_rs over every rank.  With
        // IN_PLACE the body's own fallback is pt2pt_rs over (count / n) * n elements (:4095-4100),
        // then the wrapper's pt2pt_rs on the remainder (:3800-3818): two calls, as on one node
        const int chain[2] = {PV_AR_RING_WRAPPER, PV_AR_SHM_RS};
        pvar_note_ids(chain, 2);
        const size_t main = in_place ? (count / (size_t)gsize) * (size_t)gsize : 0;
        if (main && main < count) {
            if ((rc = mn_flat_allreduce(sendbuf, recvbuf, main, dtype, op, stream, ALG_PT2PT_RS))) return rc;
            const size_t off = main * (size_t)dt->extent;
            return mn_flat_allreduce(sendbuf, (char *)recvbuf + off, count - main, dtype, op, stream, ALG_PT2PT_RS);
        }
        return mn_flat_allreduce(sendbuf, recvbuf, count, dtype, op, stream, ALG_PT2PT_RS);
    }
    if (sel == ALG_PT2PT_RS || sel == ALG_PT2PT_RD)
        return mn_flat_allreduce(sendbuf, recvbuf, count, dtype, op, stream, sel);
    return mn_allreduce_2lvl(sendbuf, recvbuf, count, dtype, op, stream, intra, inter);
}

// The node step of a two-level table entry: the entry's intra-node function over the node's ranks
// (MPIR_Allreduce_two_level_MV2 :1727-1745; the leader's result is what the leaders reduce, and the
// node broadcast that ends the call overwrites every other rank's).  MN_INTRA_NODE: the node's own
// one-node selection, which reads the same table entry (16 ppn) or is the shortcut's order.
static int node_allreduce_intra(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream,
                                int intra) {
    if (intra == MN_INTRA_NODE) return allreduce_entry(sendbuf, recvbuf, count, dtype, op, stream);
    const DtypeInfo *dt = nullptr;
    int rc = check_op_dtype(op, dtype, &dt);
    if (rc || count == 0) return rc;
    if ((rc = kind_supported(dt)) || (rc = require_world())) return rc;
    World &w = world();
    const int n = w.size, me = w.rank, oi = op_index(op);
    const bool in_place = sendbuf == (const void *)-1;
    if (n == 1 || oi == OP_NO_OP || oi == OP_REPLACE)
        return allreduce_impl(sendbuf, recvbuf, count, dt, oi, pick_stream(stream), tree_base(n));
    Plan p;
    if (intra == MN_INTRA_P2P) {  // MPIR_Reduce_MV2 to local rank 0 (the node's reduce selection)
        rc = plan_reduce(n, me, 0, count, dt->size, dt->extent, &p);
        p.inner = p.algo;
        p.algo = ALG_TWO_LEVEL_P2P;
    } else {
        rc = plan_allreduce(n, me, count, dt->size, dt->extent, in_place,
                            intra == MN_INTRA_RS   ? ALG_PT2PT_RS
                            : intra == MN_INTRA_RD ? ALG_PT2PT_RD
                                                   : ALG_SHMEM_LINEAR,
                            &p);
    }
    if (rc) return rc;
    log_plan("allreduce (node step)", p, count);
    return allreduce_impl(sendbuf, recvbuf, count, dt, oi, pick_stream(stream), tree_from_plan(p, n, count, me));
}

namespace {
// leaders: MPIR_Allreduce_pt2pt_rs_MV2 (:633-1054; recursive doubling for count < pof2, :802) with
// the nodes as ranks, MPI_IN_PLACE on `acc`.  Every leader's partial reaches every leader (a ring
// over the leaders) and each evaluates that algorithm's per-element programs for its own node
// index on the device; more than kMaxRanks nodes run the algorithm's message schedule itself.
int leader_prog(char *acc, size_t count, int dtype, int op, size_t bytes, int algo) {
    World &w = world();
    const int K = w.nnodes, me = w.node;
    if (K > mn_prog_max()) {
        LeaderLinks x;
        return sched_allreduce(x, K, me, acc, g_mn.d1, count, bytes / count, dtype, op, algo == ALG_PT2PT_RD);
    }
    const DtypeInfo *dt = dtype_lookup(dtype);
    Plan p;
    int rc = plan_allreduce(K, me, count, dt->size, dt->extent, true, algo, &p);
    if (rc) return rc;
    char *W = (char *)get_scratch(6, (size_t)K * bytes);
    if (!W) return E_NO_MEM;
    if ((rc = mn_reserve_host((size_t)K * bytes)) || (rc = mn_d2h(g_mn.h0 + (size_t)me * bytes, acc, bytes)))
        return rc;
    const int right = (me + 1) % K, left = (me - 1 + K) % K;
    for (int k = 0; k < K - 1; ++k) {
        const int so = (me - k + K) % K, ro = (me - k - 1 + K) % K;
        if ((rc = net_shift(right, g_mn.h0 + (size_t)so * bytes, bytes, left, g_mn.h0 + (size_t)ro * bytes, bytes)))
            return rc;
    }
    if ((rc = mn_h2d(W, g_mn.h0, (size_t)K * bytes))) return rc;
    const void *srcs[kMaxRanks];
    for (int r = 0; r < K; ++r) srcs[r] = W + (size_t)r * bytes;
    return mv2h_reduce_n_prog(srcs, K, acc, count, dtype, op, (const mv2h_progset *)&p.ps, nullptr);
}
}  // namespace

static int mn_allreduce_2lvl(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream,
                             int intra, int inter) {
    World &w = world();
    int rc = 0;
    const DtypeInfo *dt = dtype_lookup(dtype);
    const size_t bytes = count * (size_t)dt->extent;
    // MPI_T: MPIR_Allreduce_two_level_MV2 (allreduce_osu.c:1693) with the leaders' recursive
    // doubling (MPIR_Allreduce_pt2pt_rd_MV2 :366) or pt2pt_rs (:639); the node step's own plan is
    // not counted
    const int chain[2] = {PV_AR_2LVL, inter == ALG_PT2PT_RS ? PV_AR_SHM_RS : PV_AR_SHM_RD};
    pvar_note_ids(chain, w.rank == 0 ? 2 : 1);
    // node step: the leader holds the node's partial
    if ((rc = node_allreduce_intra(sendbuf, recvbuf, count, dtype, op, stream, intra))) return rc;
    if (w.rank == 0) {
        if ((rc = mn_reserve(bytes))) return rc;
        if ((rc = mn_h2d(g_mn.d0, recvbuf, bytes)) ||
            (rc = inter == ALG_PT2PT_RS ? leader_prog(g_mn.d0, count, dtype, op, bytes, ALG_PT2PT_RS)
                                        : leader_rd(g_mn.d0, count, dtype, op, bytes)) ||
            (rc = mn_d2h(recvbuf, g_mn.d0, bytes)))
            return rc;
    }
    return bcast_node(recvbuf, bytes, 0, stream);  // MPIR_Shmem_Bcast_MV2 from the leader
}

static int mn_bcast(void *buffer, size_t bytes, int root, void *stream) {
    World &w = world();
    if (root < 0 || root >= w.gsize) return E_ROOT;
    if (bytes == 0) return 0;
    const int rnode = root / w.size, rlocal = root % w.size;
    int rc = 0;
    if (w.node == rnode && rlocal != 0 && (rc = bcast_node(buffer, bytes, rlocal, stream))) return rc;
    if (w.rank == 0) {
        if ((rc = mn_reserve(bytes))) return rc;
        if (w.node == rnode && (rc = mn_d2h(g_mn.h0, buffer, bytes))) return rc;
        if ((rc = leader_bcast(g_mn.h0, bytes, rnode))) return rc;
        if (w.node != rnode && (rc = mn_h2d(buffer, g_mn.h0, bytes))) return rc;
    }
    if (w.node != rnode || rlocal == 0) rc = bcast_node(buffer, bytes, 0, stream);
    return rc;
}

// MPI_Reduce across nodes: the nonblocking schedule (MPI_Ireduce), else MPIR_Reduce_index_tuned_intra_MV2's
// choice (mn_reduce_select): MPIR_Reduce_two_level_helper_MV2 (reduce_osu.c:2030-2330: the node step
// to local rank 0, the leaders' algorithm to the root's node, the leader to the root) or a flat
// algorithm over every rank (programs up to kMaxRanks, its message schedule up to the rank mesh,
// the two-level helper with the shortcut's steps beyond).
static int mn_reduce_flat_sched(const void *src, void *recvbuf, size_t count, const DtypeInfo *dt, int dtype, int op,
                                int root, int algo, int k) {
    World &w = world();
    const size_t ext = (size_t)dt->extent, S = count * ext;
    const int n = w.gsize, me = w.grank;
    int rc = mn_reserve_dev(S);
    if (rc) return rc;
    const bool mine = me == root && recvbuf && is_device(recvbuf);
    char *acc = mine ? (char *)recvbuf : g_mn.d0;
    if (src != acc && hipMemcpy(acc, src, S, hipMemcpyDefault) != hipSuccess) return E_INTERN;
    RankChannels x;
    if (algo == ALG_KNOMIAL) rc = sched_knomial_reduce(x, n, me, root, k, acc, g_mn.d1, count, ext, dtype, op);
    else if (algo == ALG_REDSCAT_GATHER) rc = sched_allreduce(x, n, me, acc, g_mn.d1, count, ext, dtype, op, false, true);
    else rc = sched_binomial_reduce(x, n, me, root, acc, g_mn.d1, count, ext, dtype, op);
    if (rc || me != root || acc == recvbuf) return rc;
    return hipMemcpy(recvbuf, acc, S, hipMemcpyDefault) == hipSuccess ? 0 : E_INTERN;
}

// the leaders' step of the two-level helper: every leader's partial in g_mn.d0, the result in the
// root node's leader's g_mn.d0.  Up to kMaxRanks nodes the partials travel to that leader, which
// evaluates the algorithm's programs for the root node; above, the message schedule runs.
static int mn_reduce_leaders(size_t count, const DtypeInfo *dt, int dtype, int op, int rnode, int algo, int k) {
    World &w = world();
    const int K = w.nnodes, me = w.node;
    const size_t ext = (size_t)dt->extent, bytes = count * ext;
    int rc = 0;
    if (K > mn_prog_max()) {
        LeaderLinks x;
        if (algo == ALG_KNOMIAL) return sched_knomial_reduce(x, K, me, rnode, k, g_mn.d0, g_mn.d1, count, ext, dtype, op);
        if (algo == ALG_REDSCAT_GATHER)
            return sched_allreduce(x, K, me, g_mn.d0, g_mn.d1, count, ext, dtype, op, false, true);
        return sched_binomial_reduce(x, K, me, rnode, g_mn.d0, g_mn.d1, count, ext, dtype, op);
    }
    if (me != rnode) return (rc = mn_d2h(g_mn.h0, g_mn.d0, bytes)) ? rc : net_send(rnode, g_mn.h0, bytes);
    Plan pl;
    if ((rc = plan_reduce_forced(K, rnode, count, algo, k, &pl))) return rc;
    char *W = (char *)get_scratch(6, (size_t)K * bytes);
    if (!W) return E_NO_MEM;
    for (int j = 0; j < K; ++j) {
        if (j == me) rc = hipMemcpy(W + (size_t)j * bytes, g_mn.d0, bytes, hipMemcpyDeviceToDevice) == hipSuccess ? 0 : E_INTERN;
        else if (!(rc = net_recv(j, g_mn.h1, bytes))) rc = mn_h2d(W + (size_t)j * bytes, g_mn.h1, bytes);
        if (rc) return rc;
    }
    const void *srcs[kMaxRanks];
    for (int j = 0; j < K; ++j) srcs[j] = W + (size_t)j * bytes;
    return mv2h_reduce_n_prog(srcs, K, g_mn.d0, count, dtype, op, (const mv2h_progset *)&pl.ps, nullptr);
}

static int mn_reduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, int root, void *stream) {
    World &w = world();
    if (root < 0 || root >= w.gsize) return E_ROOT;
    int rc = mn_require_device_reduction(dtype, op);
    if (rc || count == 0) return rc;
    const DtypeInfo *dt = dtype_lookup(dtype);
    const size_t bytes = count * (size_t)dt->extent;
    const int rnode = root / w.size, rlocal = root % w.size;
    const bool me_root = w.grank == root;
    const void *src = sendbuf == (const void *)-1 ? recvbuf : sendbuf;  // IN_PLACE: at the root only
    // MPI_Ireduce: MVAPICH2's nonblocking schedule (MPIR_Ireduce_binomial, ireduce_osu.c) is flat
    // over the whole job
    if (nbc_kind() == NBC_IREDUCE) {
        const int route = mn_flat_route(w.gsize);
        if (route == MN_FLAT_PROG) return mn_flat_allreduce(sendbuf, recvbuf, count, dtype, op, stream, 0, root);
        if (route == MN_SCHED) return mn_sched_naive(sendbuf, recvbuf, count, dtype, op, stream, root);
    }
    MnRedSel sel = mn_reduce_select(w.size, w.gsize, count, dt->size, dt->extent, OPK_BUILTIN);
    if (nbc_kind() == NBC_IREDUCE || (!sel.two_level && mn_flat_route(w.gsize) == MN_FALLBACK))
        sel = MnRedSel{true, ALG_SHMEM_LINEAR, ALG_BINOMIAL, sel.k};  // beyond the rank mesh (unpinned)
    if (!sel.two_level) {
        const int ids[3] = {sel.algo == ALG_KNOMIAL ? PV_RED_KNOMIAL : sel.algo == ALG_REDSCAT_GATHER ? PV_RED_REDSCAT_GATHER
                                                                                                       : PV_RED_BINOMIAL};
        pvar_note_ids(ids, 1);
        if (mn_flat_route(w.gsize) == MN_FLAT_PROG) {
            Plan p;
            if ((rc = plan_reduce_forced(w.gsize, root, count, sel.algo, sel.k, &p))) return rc;
            return mn_flat_allreduce(sendbuf, recvbuf, count, dtype, op, stream, 0, root, &p);
        }
        return mn_reduce_flat_sched(src, recvbuf, count, dt, dtype, op, root, sel.algo, sel.k);
    }
    // MPIR_Reduce_two_level_helper_MV2 (reduce_osu.c:2039) with the leaders' function
    const int chain[2] = {PV_RED_TWO_LEVEL_HELPER, sel.algo == ALG_KNOMIAL ? PV_RED_KNOMIAL
                                                   : sel.algo == ALG_REDSCAT_GATHER ? PV_RED_REDSCAT_GATHER
                                                                                    : PV_RED_BINOMIAL};
    pvar_note_ids(chain, w.rank == 0 && w.nnodes > 1 ? 2 : 1);
    if ((rc = mn_reserve_dev(bytes)) || (w.rank == 0 && (rc = mn_reserve_host(bytes)))) return rc;
    // node step to local rank 0: the leader's partial lands in g_mn.d0 (a non-root's recvbuf is not
    // significant)
    if (w.size > 1) {
        Plan pn;
        if ((rc = plan_reduce_forced(w.size, 0, count, sel.intra, sel.k, &pn)) ||
            (rc = reduce_entry(src, w.rank == 0 ? g_mn.d0 : nullptr, count, dtype, op, 0, stream, &pn)))
            return rc;
    } else if (hipMemcpy(g_mn.d0, src, bytes, hipMemcpyDefault) != hipSuccess) {
        return E_INTERN;
    }
    if (w.rank == 0 && (rc = mn_reduce_leaders(count, dt, dtype, op, rnode, sel.algo, sel.k))) return rc;
    if (w.node != rnode) return 0;
    if (rlocal == 0) return me_root ? mn_d2h(recvbuf, g_mn.d0, bytes) : 0;
    // the root is not the leader: the node's device point-to-point channel carries the result
    unsigned long long req = 0;
    if (w.rank == 0) {
        if ((rc = p2p_isend(g_mn.d0, bytes, root, kCollTagBase - 1, &req))) return rc;
        return mv2h_p2p_wait(req, nullptr, nullptr, nullptr);
    }
    if (me_root) {
        if ((rc = p2p_irecv(recvbuf, bytes, w.node * w.size, kCollTagBase - 1, &req))) return rc;
        return mv2h_p2p_wait(req, nullptr, nullptr, nullptr);
    }
    return 0;
}

static int mn_allgather(const void *sendbuf, void *recvbuf, size_t bytes, void *stream) {
    World &w = world();
    if (bytes == 0) return 0;
    const size_t sect = bytes * (size_t)w.size, total = sect * (size_t)w.nnodes;
    char *mine = (char *)recvbuf + (size_t)w.node * sect;
    const bool in_place = sendbuf == (const void *)-1;
    int rc = allgather_node(in_place ? (const void *)(mine + (size_t)w.rank * bytes) : sendbuf, mine, bytes, stream);
    if (rc) return rc;
    if (w.rank == 0) {
        if ((rc = mn_reserve(total))) return rc;
        if ((rc = mn_d2h(g_mn.h0 + (size_t)w.node * sect, mine, sect))) return rc;
        // ring over the leaders: step k passes node (node - k)'s section to the right
        const int n = w.nnodes, right = (w.node + 1) % n, left = (w.node - 1 + n) % n;
        for (int k = 0; k < n - 1; ++k) {
            const int so = (w.node - k + n) % n, ro = (w.node - k - 1 + n) % n;
            if ((rc = net_shift(right, g_mn.h0 + (size_t)so * sect, sect, left, g_mn.h0 + (size_t)ro * sect, sect)))
                return rc;
        }
        if ((rc = mn_h2d(recvbuf, g_mn.h0, total))) return rc;
    }
    return bcast_node(recvbuf, total, 0, stream);
}

// Reduce_scatter across nodes: MPIR_Reduce_scatter_MV2 runs its flat algorithms over every rank of
// the job (red_scat_osu.c:1771-1900: ring / basic / recursive halving / pairwise by total size, the
// non-commutative forms for non-commutative ops; MPI_Ireduce_scatter: pairwise).  Every operand
// reaches every rank (mn_gather_all) and each rank evaluates its own block's programs of the
// selected algorithm over the job's ranks (orders.cpp plan_reduce_scatter, the same restatement as
// on one node).  Jobs above kMaxRanks ranks: the algorithm's message schedule itself
// (sched_rs_halving / _pairwise / _ring over the rank channels).  The basic algorithm at any size
// is MPIR_Reduce_MV2 over the whole job (the multi-node reduce) and a scatter.
static int mn_reduce_scatter(const void *sendbuf, void *recvbuf, const size_t *recvcounts, int dtype, int op,
                             void *stream) {
    World &w = world();
    int rc = mn_require_device_reduction(dtype, op);
    if (rc) return rc;
    const DtypeInfo *dt = dtype_lookup(dtype);
    size_t total = 0, off = 0;
    for (int j = 0; j < w.gsize; ++j) {
        if (j == w.grank) off = total;
        total += recvcounts[j];
    }
    if (total == 0) return 0;
    const size_t ext = (size_t)dt->extent, S = total * ext;
    const bool in_place = sendbuf == (const void *)-1;
    const void *src = in_place ? recvbuf : sendbuf;
    const int n = w.gsize, me = w.grank, oi = op_index(op);
    const size_t mine = recvcounts[me] * ext;
    if (oi == OP_NO_OP || oi == OP_REPLACE) {  // nothing to reduce: this rank's own block
        return !mine || hipMemcpy(recvbuf, (const char *)src + off * ext, mine, hipMemcpyDefault) == hipSuccess
                   ? 0 : E_INTERN;
    }
    const int algo = reduce_scatter_algo(n, (long)(total * (size_t)dt->size));
    const int route = mn_reduce_scatter_route(n, (long)(total * (size_t)dt->size));
    if (route == MN_BASIC_R) {
        // MPIR_Reduce_Scatter_Basic_MV2 (red_scat_osu.c:300-413): MPIR_Reduce_MV2 to rank 0 over
        // the whole communicator — the multi-node reduce (mn_reduce) — then the blocks scattered
        const int chain[3] = {PV_RS_BASIC, PV_RED_TWO_LEVEL_HELPER, PV_RED_BINOMIAL};
        pvar_note_ids(chain, w.rank == 0 ? 3 : 2);
        char *tmp = (char *)get_scratch(5, S);
        if (!tmp) return E_NO_MEM;
        if ((rc = mn_reduce(src, tmp, total, dtype, op, 0, stream)) || (rc = mn_bcast(tmp, S, 0, stream))) return rc;
        return !mine || hipMemcpy(recvbuf, tmp + off * ext, mine, hipMemcpyDefault) == hipSuccess ? 0 : E_INTERN;
    }
    if (route == MN_SCHED) {
        // beyond the programs' registers: the algorithm's message schedule over the rank channels
        const int id = algo == ALG_RS_RING ? PV_RS_RING : algo == ALG_RS_PAIRWISE ? PV_RS_PAIRWISE : PV_RS_REC_HALVING;
        pvar_note_ids(&id, 1);
        std::vector<size_t> disps((size_t)n, 0);
        for (int j = 1; j < n; ++j) disps[j] = disps[j - 1] + recvcounts[j - 1];
        if ((rc = mn_reserve_dev(S))) return rc;
        const char *in = (const char *)src;
        if (!is_device(src)) {  // a host operand: staged to the device once
            char *stage = (char *)get_scratch(5, S);
            if (!stage || hipMemcpy(stage, src, S, hipMemcpyDefault) != hipSuccess) return stage ? E_INTERN : E_NO_MEM;
            in = stage;
        }
        // (MPI_IN_PLACE needs no copy: every schedule writes this rank's block after its last read)
        RankChannels x;
        auto fn = algo == ALG_RS_RING ? sched_rs_ring : algo == ALG_RS_PAIRWISE ? sched_rs_pairwise : sched_rs_halving;
        return fn(x, n, me, recvcounts, disps.data(), in, (char *)recvbuf, g_mn.d0, g_mn.d1, ext, dtype, op);
    }
    Plan p;
    if ((rc = plan_reduce_scatter(w.gsize, w.grank, recvcounts, dt->size, dt->extent, &p))) return rc;
    log_plan("reduce_scatter (flat over the job)", p, total);
    pvar_note(PV_COLL_REDUCE_SCATTER, p, in_place, total, w.gsize);
    char *W = nullptr;
    if ((rc = mn_reserve_dev(S)) || (rc = mn_gather_all(src, S, &W, stream))) return rc;
    if (!recvcounts[w.grank]) return 0;
    const void *srcs[kMaxRanks];
    for (int r = 0; r < w.gsize; ++r) srcs[r] = W + (size_t)r * S;
    if ((rc = mv2h_reduce_n_prog(srcs, w.gsize, g_mn.d1, total, dtype, op, (const mv2h_progset *)&p.ps, nullptr)))
        return rc;
    return hipMemcpy(recvbuf, g_mn.d1 + off * ext, recvcounts[w.grank] * ext, hipMemcpyDefault) == hipSuccess
               ? 0 : E_INTERN;
}

}  // extern "C" (a C++ entry point for mpi/user_coll.cpp)

// Host-evaluated reductions across nodes (user ops, x87 types; mpi/user_coll.cpp): the schedule the
// device path above runs, as programs.  Allreduce: a non-commutative op fails every shortcut and
// every two-level test and runs recursive doubling over the job (allreduce_osu.c:3359-3368);
// MPI_Iallreduce the flat naive schedule; else mn_select's choice (flat ring wrapper / flat
// pt2pt_rs or _rd / two-level with the entry's intra and inter functions).  Reduce: the flat
// binomial for a non-commutative op (the two-level helper needs a commutative one,
// reduce_osu.c:2628-2636) and for MPI_Ireduce, else the two-level helper (node reduce to local rank
// 0, binomial over the leaders to the root's node).  Flat schedules take the job's ranks as
// program registers up to kMaxRanks; above, `big` names the schedule the host evaluates itself.
int mv2::mn_host_schedule(int coll, size_t count, int tsize, int textent, bool in_place, int opk, int root, MnSched *s) {
    const World &w = world();
    const int n = w.gsize, me = w.grank, L = w.size, K = w.nnodes;
    memset(s, 0, sizeof(*s));
    s->kind = MN_FLAT;
    s->coll = coll;
    s->U = 0;
    const bool big = n > mn_prog_max();
    int rc = 0;
    if (coll == MN_COLL_REDUCE) {
        if (opk == OPK_USER_NONCOMM || nbc_kind() == NBC_IREDUCE) {
            if (big) {  // the flat binomial (MPIR_Reduce_binomial_MV2 / MPIR_Ireduce_binomial)
                const int id = PV_RED_BINOMIAL;
                if (nbc_kind() == NBC_NONE) pvar_note_ids(&id, 1);
                s->big = 1;
                s->forced = ALG_BINOMIAL;
                s->root = root;
                return 0;
            }
            rc = plan_reduce(n, me, root, count, tsize, textent, &s->p, opk);
            if (!rc) pvar_note(PV_COLL_REDUCE, s->p, in_place, count, n);
            return rc;
        }
        // MPIR_Reduce_index_tuned_intra_MV2's choice across nodes, as on the device path (mn_reduce)
        const MnRedSel sel = mn_reduce_select(L, n, count, tsize, textent, opk);
        const int fid = sel.algo == ALG_KNOMIAL ? PV_RED_KNOMIAL : sel.algo == ALG_REDSCAT_GATHER ? PV_RED_REDSCAT_GATHER
                                                                                                 : PV_RED_BINOMIAL;
        s->k = sel.k;
        if (!sel.two_level) {
            pvar_note_ids(&fid, 1);
            if (big) {  // the flat algorithm's schedule, evaluated on the host
                s->big = 1;
                s->forced = sel.algo;
                s->root = root;
                return 0;
            }
            s->forced = sel.algo;
            return plan_reduce_forced(n, root, count, sel.algo, sel.k, &s->p);
        }
        s->kind = MN_TWO_LEVEL;
        const int chain[2] = {PV_RED_TWO_LEVEL_HELPER, fid};
        pvar_note_ids(chain, w.rank == 0 ? 2 : 1);
        if ((rc = plan_reduce_forced(L, 0, count, sel.intra, sel.k, &s->node))) return rc;
        if (K > mn_prog_max()) {
            s->big = 1;
            s->forced = sel.algo;
            s->root = root / L;
            return 0;
        }
        return plan_reduce_forced(K, root / L, count, sel.algo, sel.k, &s->lead);
    }
    if (big && nbc_kind() == NBC_IALLREDUCE) {
        // MPIR_Iallreduce_naive: Ireduce to rank 0 — binomial for a user op (redscat_gather needs a
        // builtin one, ireduce.c:700-731) — and Ibcast: every rank takes rank 0's result
        s->big = 1;
        s->forced = ALG_BINOMIAL;
        s->root = 0;
        return 0;
    }
    if (big && opk == OPK_USER_NONCOMM) {  // every shortcut and two-level test fails: recursive doubling
        const int id = PV_AR_SHM_RD;
        pvar_note_ids(&id, 1);
        s->big = 1;
        s->forced = ALG_PT2PT_RD;
        return 0;
    }
    if (opk == OPK_USER_NONCOMM || nbc_kind() == NBC_IALLREDUCE) {
        if ((rc = plan_allreduce(n, me, count, tsize, textent, in_place, 0, &s->p, opk))) return rc;
        pvar_note(PV_COLL_ALLREDUCE, s->p, in_place, count, n);
        return 0;
    }
    int intra = MN_INTRA_NODE, inter = ALG_PT2PT_RD;
    const int sel = mn_select(L, n, (long)count * tsize, &intra, &inter);
    if (big && sel != 0) {
        // flat over more ranks than a program holds: the ring over (count / n) * n elements unless
        // IN_PLACE or count < n, then pt2pt_rs on the rest; IN_PLACE: two pt2pt_rs calls split
        // at (count / n) * n (:4095, :3800); else the tables' pt2pt_rs / pt2pt_rd.  (pt2pt_rs is
        // recursive doubling for a user op or fewer elements than pof2, :802.)
        s->big = 1;
        if (sel == 1 && !in_place && count >= (size_t)n) {
            const int chain[3] = {PV_AR_RING_WRAPPER, PV_AR_RING, PV_AR_SHM_RS};
            pvar_note_ids(chain, count % (size_t)n ? 3 : 2);
            s->forced = ALG_RING;
            s->U = (long)(count / n) * n;
        } else if (sel == 1) {
            const int chain[2] = {PV_AR_RING_WRAPPER, PV_AR_SHM_RS};
            pvar_note_ids(chain, 2);
            s->forced = ALG_PT2PT_RS;
            s->U = in_place ? (long)(count / n) * n : 0;
            if ((size_t)s->U == count) s->U = 0;
        } else {
            const int id = sel == ALG_PT2PT_RS || opk != OPK_BUILTIN ? PV_AR_SHM_RS : PV_AR_SHM_RD;
            pvar_note_ids(&id, 1);
            s->forced = sel;
        }
        return 0;
    }
    if (sel == 1 && n <= mn_prog_max()) {  // the flat ring wrapper over every rank
        const int chain[3] = {PV_AR_RING_WRAPPER, PV_AR_RING, PV_AR_SHM_RS};
        if (!in_place && count >= (size_t)n) {
            pvar_note_ids(chain, count % (size_t)n ? 3 : 2);
            s->forced = ALG_RING;
            s->U = (long)(count / n) * n;
            if ((rc = plan_allreduce(n, me, (size_t)s->U, tsize, textent, false, ALG_RING, &s->p, opk))) return rc;
        } else {
            const int rs_chain[2] = {PV_AR_RING_WRAPPER, PV_AR_SHM_RS};
            pvar_note_ids(rs_chain, 2);
            s->forced = ALG_PT2PT_RS;
            s->U = in_place ? (long)(count / n) * n : 0;  // IN_PLACE: two pt2pt_rs calls (:4095, :3800)
            if (s->U && (rc = plan_allreduce(n, me, (size_t)s->U, tsize, textent, true, ALG_PT2PT_RS, &s->p, opk)))
                return rc;
        }
        if ((size_t)s->U < count)
            rc = plan_allreduce(n, me, count - (size_t)s->U, tsize, textent, in_place, ALG_PT2PT_RS, &s->rem, opk);
        if (!s->U) s->p = s->rem;
        return rc;
    }
    if ((sel == ALG_PT2PT_RS || sel == ALG_PT2PT_RD) && n <= mn_prog_max()) {
        s->forced = sel;
        if ((rc = plan_allreduce(n, me, count, tsize, textent, in_place, sel, &s->p, opk))) return rc;
        pvar_note(PV_COLL_ALLREDUCE, s->p, in_place, count, n);
        return 0;
    }
    s->kind = MN_TWO_LEVEL;
    const int chain[2] = {PV_AR_2LVL, inter == ALG_PT2PT_RS ? PV_AR_SHM_RS : PV_AR_SHM_RD};
    pvar_note_ids(chain, w.rank == 0 ? 2 : 1);
    switch (intra) {
    case MN_INTRA_P2P: rc = plan_reduce(L, 0, 0, count, tsize, textent, &s->node, opk); break;
    case MN_INTRA_SHMEM: rc = plan_allreduce(L, 0, count, tsize, textent, in_place, ALG_SHMEM_LINEAR, &s->node, opk); break;
    case MN_INTRA_RS: rc = plan_allreduce(L, 0, count, tsize, textent, in_place, ALG_PT2PT_RS, &s->node, opk); break;
    case MN_INTRA_RD: rc = plan_allreduce(L, 0, count, tsize, textent, in_place, ALG_PT2PT_RD, &s->node, opk); break;
    default: rc = plan_allreduce(L, 0, count, tsize, textent, in_place, 0, &s->node, opk); break;
    }
    if (rc) return rc;
    if (K > mn_prog_max()) {  // the leaders' pt2pt_rs / _rd: recursive doubling for a user op
        s->big = 1;
        s->forced = ALG_PT2PT_RD;
        return 0;
    }
    return plan_allreduce(K, w.node, count, tsize, textent, true, inter, &s->lead, opk);
}

extern "C" {

int mv2h_rs_noncomm_expr(int n, int me, int pof2_equal, int *leaf, int *a, int *b, int cap, int *root) {
    if (n < 1 || me < 0 || me >= n || !root) return E_ARG;
    std::vector<ExprNode> nodes;
    *root = rs_noncomm_expr(n, me, pof2_equal != 0, nodes);
    if ((int)nodes.size() > cap || !leaf || !a || !b) return -(int)nodes.size();
    for (size_t i = 0; i < nodes.size(); ++i) {
        leaf[i] = nodes[i].leaf;
        a[i] = nodes[i].a;
        b[i] = nodes[i].b;
    }
    return (int)nodes.size();
}

int mv2h_mn_reduce_table(int ppn, int gsize, long nbytes, int *two_level, int *inter, int *intra, int *k) {
    if (ppn < 1 || gsize < 1) return E_ARG;
    MnReduceCell c{};
    const int rc = mn_reduce_table(ppn, gsize, nbytes, &c);
    if (two_level) *two_level = c.two_level;
    if (inter) *inter = c.inter;
    if (intra) *intra = c.intra;
    if (k) *k = c.k;
    return rc ? rc : c.entry;
}

int mv2h_mn_route(int coll, int ppn, int gsize, long nbytes, size_t count, int in_place, int nbc, int *rem_route) {
    if (ppn < 1 || gsize < ppn || gsize % ppn) return E_ARG;
    int intra = 0, inter = 0, sel = 0, rem = -1;
    int r;
    switch (coll) {
    case 0: r = mn_allreduce_route(ppn, gsize, nbytes, count, in_place != 0, nbc, &intra, &inter, &sel, &rem); break;
    case 1: r = mn_reduce_route(ppn, gsize, count, nbytes > 0 && count ? (int)(nbytes / (long)count) : 4, nbc); break;
    case 2: r = mn_reduce_scatter_route(gsize, nbytes); break;
    default: return E_ARG;
    }
    if (rem_route) *rem_route = rem;
    return r;
}

int mv2h_allgather(const void *sendbuf, void *recvbuf, size_t bytes, void *stream) {
    if (world().nnodes > 1) {
        int rc0 = 0;
        if (world().enqueue && (rc0 = mn_stream_order(&stream))) return rc0;
        MnBlocking nb;
        return mn_allgather(sendbuf, recvbuf, bytes, stream);
    }
    return allgather_node(sendbuf, recvbuf, bytes, stream);
}

int mv2h_bcast(void *buffer, size_t bytes, int root, void *stream) {
    if (world().nnodes > 1) {
        int rc0 = 0;
        if (world().enqueue && (rc0 = mn_stream_order(&stream))) return rc0;
        MnBlocking nb;
        return mn_bcast(buffer, bytes, root, stream);
    }
    return bcast_node(buffer, bytes, root, stream);
}

// ---------------------------------------------------------------------------
// part (3): strided pack / unpack
// ---------------------------------------------------------------------------
int mv2h_pack_strided(const void *src, void *dst, size_t nblocks, size_t blk, size_t stride, void *stream) {
    hp_entry();  // a new API call: the timing events bracket its own launches
    int rc;
    if ((rc = ensure_init_for_device())) return rc;
    hipStream_t st = pick_stream(stream);
    tmark0(st);
    rc = launch_pack_strided(src, dst, nblocks, blk, stride, 0, st, arm_done(st));
    tmark1(st);
    if (rc) return rc;
    return finish(st, world().timing);
}

int mv2h_unpack_strided(const void *src, void *dst, size_t nblocks, size_t blk, size_t stride, void *stream) {
    hp_entry();  // a new API call: the timing events bracket its own launches
    int rc;
    if ((rc = ensure_init_for_device())) return rc;
    hipStream_t st = pick_stream(stream);
    tmark0(st);
    rc = launch_pack_strided(src, dst, nblocks, blk, stride, 1, st, arm_done(st));
    tmark1(st);
    if (rc) return rc;
    return finish(st, world().timing);
}

int mv2h_pack_segments(const void *src, void *dst, size_t count, size_t extent, const int64_t *offs,
                       const int64_t *lens, int nseg, int unpack, void *stream) {
    hp_entry();  // a new API call: the timing events bracket its own launches
    int rc;
    if ((rc = ensure_init_for_device())) return rc;
    hipStream_t st = pick_stream(stream);
    tmark0(st);
    rc = launch_pack_runs(src, dst, count, extent, offs, lens, nseg, unpack ? 1 : 0, st, arm_done(st));
    tmark1(st);
    if (rc) return rc;
    return finish(st, world().timing);
}

// ---------------------------------------------------------------------------
// Stream-ordered collectives (§8(f) rank 3, "stream-ordered variants"): the same selection,
// orders and kernels as the blocking calls, launched on the caller's HIP stream after every
// collective this process issued before (pick_stream), returning without waiting.  Kernels
// queued behind it on that stream see the result; the host never blocks, so compute and
// communication overlap without MPI_Wait.  Device buffers only (a host buffer would need a
// host copy after the kernel) and builtin ops (user ops and x87 run on the host).
// ---------------------------------------------------------------------------
struct EnqueueScope {
    explicit EnqueueScope(bool graph = false) {
        world().enqueue = true;
        world().graph = graph;
    }
    ~EnqueueScope() {
        world().enqueue = false;
        world().graph = false;
    }
};
static bool capturing(void *stream) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return stream && hipStreamIsCapturing((hipStream_t)stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
static int enqueue_checks(const void *send, const void *recv, void *stream, bool graph_ok = false) {
    if (!stream) return E_ARG;
    // a destroyed stream or one of another device is an argument error, not a launch into it
    int sdev = -1;
    if (hipStreamGetDevice((hipStream_t)stream, &sdev) != hipSuccess || sdev != world().device) {
        (void)hipGetLastError();
        MV2_ERR("stream-ordered call: the stream is not a live stream of this rank's device");
        return E_ARG;
    }
    // host-managed epochs and parities would be replayed by a graph: a captured call must take
    // the graph lane (allreduce on 16-byte-aligned device buffers), anything else is refused
    if (capturing(stream)) {
        const World &w = world();
        if (!graph_ok || !w.graph_lane || w.size < 2 || w.nnodes > 1) {
            MV2_ERR("only collectives on one node can be captured into a HIP graph (graph lane %s)",
                    w.graph_lane ? "on" : "off");
            return E_UNSUPPORTED;
        }
        if ((uintptr_t)recv % 16 || (send && send != (const void *)-1 && (uintptr_t)send % 16)) {
            MV2_ERR("a captured collective needs 16-byte-aligned buffers");
            return E_ARG;
        }
    }
    if (!is_device(recv) || (send && send != (const void *)-1 && !is_device(send))) {
        MV2_ERR("stream-ordered collectives take device buffers only");
        return E_ARG;
    }
    return 0;
}

int mv2h_allreduce_enqueue(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, void *stream) {
    int rc = count ? enqueue_checks(sendbuf, recvbuf, stream, true) : 0;
    if (rc || !count) return rc;
    const bool graph = capturing(stream);
    if (graph && op_index(op) >= OP_REPLACE) return E_OP;
    EnqueueScope q(graph);
    return mv2h_allreduce(sendbuf, recvbuf, count, dtype, op, stream);
}

int mv2h_reduce_enqueue(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, int root, void *stream) {
    if (!count) return 0;
    const World &w = world();
    // recvbuf is significant at the root only
    int rc = enqueue_checks(sendbuf, w.grank == root ? recvbuf : (sendbuf == (const void *)-1 ? nullptr : sendbuf),
                            stream, true);
    if (rc) return rc;
    const bool graph = capturing(stream);
    if (graph && op_index(op) >= OP_REPLACE) return E_OP;  // those run as a broadcast after a host wait
    EnqueueScope q(graph);
    return mv2h_reduce(sendbuf, recvbuf, count, dtype, op, root, stream);
}

int mv2h_reduce_scatter_enqueue(const void *sendbuf, void *recvbuf, const size_t *recvcounts, int dtype, int op,
                                void *stream) {
    const World &w = world();
    if (!recvcounts) return E_ARG;
    int rc = enqueue_checks(sendbuf, recvcounts[w.rank] ? recvbuf : (sendbuf == (const void *)-1 ? nullptr : sendbuf),
                            stream, true);
    if (rc) return rc;
    EnqueueScope q(capturing(stream));
    return mv2h_reduce_scatter(sendbuf, recvbuf, recvcounts, dtype, op, stream);
}

int mv2h_allgather_enqueue(const void *sendbuf, void *recvbuf, size_t bytes, void *stream) {
    int rc = bytes ? enqueue_checks(sendbuf, recvbuf, stream, true) : 0;
    if (rc || !bytes) return rc;
    EnqueueScope q(capturing(stream));
    return mv2h_allgather(sendbuf, recvbuf, bytes, stream);
}

int mv2h_bcast_enqueue(void *buffer, size_t bytes, int root, void *stream) {
    int rc = bytes ? enqueue_checks(nullptr, buffer, stream, true) : 0;
    if (rc || !bytes) return rc;
    EnqueueScope q(capturing(stream));
    return mv2h_bcast(buffer, bytes, root, stream);
}

// device-to-device copy in the same stream order (COMM_SELF forms of the calls above)
int mv2h_copy_enqueue(void *dst, const void *src, size_t bytes, void *stream) {
    int rc = bytes ? enqueue_checks(src, dst, stream) : 0;
    if (rc || !bytes) return rc;
    if ((rc = ensure_init_for_device())) return rc;
    hipStream_t st = pick_stream(stream);
    rc = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st) == hipSuccess ? 0 : E_INTERN;
    stream_tail(st);
    return rc;
}

// errors of stream-ordered calls (a peer that never arrived) surface once their stream has
// been synchronised: the kernels set the host error word instead of hanging
int mv2h_enqueue_check(void) { return check_err_word(); }

}  // extern "C"

// ===========================================================================
// MPI_Init self-test of the cross-GPU publish protocol on this node's topology
// ===========================================================================
namespace mv2 {

// The one-shot and pipelined kernels publish arena stores with the light release (stores
// acknowledged, no L2 writeback) and read them with the light acquire, which is right only if a
// peer-mapped uncached arena is not write-back cached by its writer -- a property of the links
// that the one-GPU box cannot show.  A rare ordering failure would not show in one call either, so
// MPI_Init runs every kernel that crosses GPUs, over both slot parities / arena halves, with a
// new operand pattern per call (an element of a stale slot never matches), and checks every
// element of every result on the device:
//   one-shot allreduce (6 sizes x 2 halves), one-shot reduce-scatter (3 x 2), pipelined allreduce
//   (ring order, 4 MiB, x 4; butterfly order x 2; ring + remainder), a multi-round pipelined
//   allreduce (small rounds: both parities inside one call) x 2, pipelined reduce-scatter,
//   allgather and broadcast x 2 each, one-shot allgather and broadcast x 2 each, and, with the
//   graph lane, a captured one-shot and a captured pipelined allreduce replayed 3 times each (its
//   own arenas and device sequence).
// The per-call mismatch counts are read once at the end; the verdict is agreed through the
// host control segment.  On a mismatch every rank falls back to the full system-scope release
// and runs the whole set again; a second failure fails MPI_Init instead of returning wrong
// sums later.  (Protocol contract: device_util.h:1-13.)
int coll_selftest() {
    World &w = world();
    const int n = w.size, me = w.rank;
    const int MPI_INT_H = 0x4c000405, MPI_SUM_H = 0x58000003;
    // elements per buffer: the largest checked call (1 Mi + 3 elements, a 1 Mi-element allgather
    // result) and the graph lane's second capture, which runs 8192 elements into the buffers
    constexpr size_t kGraphOff = 8192;
    const size_t cap = kGraphOff + ((size_t)1 << 20) + 64;
    constexpr int kMaxCalls = 96;
    uint32_t *sb = nullptr, *rb = nullptr, *bad = nullptr;
    if (hipMalloc((void **)&sb, cap * 4) != hipSuccess || hipMalloc((void **)&rb, cap * 4) != hipSuccess ||
        hipMalloc((void **)&bad, kMaxCalls * 4) != hipSuccess) {
        MV2_ERR("self-test: device allocation failed");
        if (sb) hipFree(sb);
        if (rb) hipFree(rb);
        return E_NO_MEM;
    }
    hipStream_t st = w.stream;
    const char *what[kMaxCalls] = {};
    int verdict = 0, calls = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        hipMemsetAsync(bad, 0, kMaxCalls * 4, st);
        int rc = 0;
        calls = 0;
        auto seed_of = [&](int k) { return (uint32_t)(0x51ed270bu * (uint32_t)(k + 1) + 0x1000193u * (uint32_t)attempt); };
        // one checked call: fill this rank's operand, run the call, check its result on the device
        // every operand and result stays inside its buffer (the graph lane's second
        // capture once ran 8 K elements past the end)
        auto fits = [&](const uint32_t *p, size_t c) {
            const uint32_t *b = (p >= rb && p < rb + cap) ? rb : sb;
            if (p < b || (size_t)(p - b) + c > cap || calls > kMaxCalls) {
                MV2_ERR("self-test: call %d does not fit its buffers (%zu elements at +%td of %zu)", calls, c, p - b, cap);
                if (!rc) rc = E_INTERN;
                return false;
            }
            return true;
        };
        auto fill = [&](uint32_t *p, size_t c, int k, int as_rank) {
            if (!rc && fits(p, c)) rc = launch_selftest_fill(p, c, seed_of(k), as_rank, st);
        };
        auto check = [&](const uint32_t *p, size_t c, int k, int mode, int arg, uint64_t base, const char *name) {
            if (!rc && fits(p, c)) rc = launch_selftest_check(p, c, seed_of(k), n, mode, arg, base, bad + k, st);
            what[k] = name;
        };
        // one-shot allreduce: sizes up to the one-shot limit, each on both arena halves
        const size_t os_max = std::min(w.oneshot_max, w.slot_bytes) / 4;
        const size_t os_sizes[6] = {2, 1027, 4096, 16389, os_max > 3 ? os_max - 3 : 1, os_max};
        for (int i = 0; i < 6 && !rc; ++i)
            for (int h = 0; h < 2 && !rc; ++h) {
                const int k = calls++;
                const size_t c = std::max<size_t>(1, std::min(os_sizes[i], cap));
                fill(sb, c, k, me);
                if (!rc) rc = ::allreduce_entry(sb, rb, c, MPI_INT_H, MPI_SUM_H, nullptr);
                check(rb, c, k, 0, 0, 0, "one-shot allreduce");
            }
        // one-shot reduce-scatter below the ring threshold: 12-byte blocks (element by element),
        // blocks of 16-byte multiples
        const size_t rs_small[3] = {3, 1024, 2048};
        for (int i = 0; i < 3 && !rc; ++i)
            for (int h = 0; h < 2 && !rc; ++h) {
                const int k = calls++;
                const size_t c = rs_small[i];
                size_t counts[kMaxRanks];
                for (int j = 0; j < n; ++j) counts[j] = c;
                fill(sb, c * n, k, me);
                if (!rc) rc = ::reduce_scatter_entry(sb, rb, counts, MPI_INT_H, MPI_SUM_H, nullptr);
                check(rb, c, k, 0, 0, (uint64_t)me * c, "one-shot reduce-scatter");
            }
        // pipelined allreduce: ring order (4 MiB) on both slot parities twice, the butterfly
        // (pt2pt_rs, 1 MiB + 5), the ring with a remainder (4 MiB + 3)
        const size_t pa_sizes[7] = {(size_t)1 << 20, (size_t)1 << 20, (size_t)1 << 20, (size_t)1 << 20,
                                    ((size_t)1 << 18) + 5, ((size_t)1 << 18) + 5, ((size_t)1 << 20) + 3};
        for (int i = 0; i < 7 && !rc; ++i) {
            const int k = calls++;
            fill(sb, pa_sizes[i], k, me);
            if (!rc) rc = ::allreduce_entry(sb, rb, pa_sizes[i], MPI_INT_H, MPI_SUM_H, nullptr);
            check(rb, pa_sizes[i], k, 0, 0, 0, "pipelined allreduce");
        }
        // multi-round pipelined allreduce: small rounds, so one call alternates slot parities
        {
            const int g0 = w.pipe_grid;
            const size_t s0 = w.pipe_sub;
            w.pipe_grid = std::min(g0, 32);
            w.pipe_sub = 4096;
            for (int i = 0; i < 2 && !rc; ++i) {
                const int k = calls++;
                const size_t c = ((size_t)1 << 20) - 7 * (size_t)i;
                fill(sb, c, k, me);
                if (!rc) rc = ::allreduce_entry(sb, rb, c, MPI_INT_H, MPI_SUM_H, nullptr);
                check(rb, c, k, 0, 0, 0, "multi-round pipelined allreduce");
            }
            w.pipe_grid = g0;
            w.pipe_sub = s0;
        }
        // pipelined reduce-scatter (ring, 4 MiB in all), allgather, broadcast
        for (int i = 0; i < 2 && !rc; ++i) {
            const int k = calls++;
            const size_t c = ((size_t)1 << 20) / (size_t)n;
            size_t counts[kMaxRanks];
            for (int j = 0; j < n; ++j) counts[j] = c;
            fill(sb, c * n, k, me);
            if (!rc) rc = ::reduce_scatter_entry(sb, rb, counts, MPI_INT_H, MPI_SUM_H, nullptr);
            check(rb, c, k, 0, 0, (uint64_t)me * c, "pipelined reduce-scatter");
        }
        // the pipelined allgather and broadcast below run with the one-shot path off: with a 1 MiB
        // slot their blocks would otherwise fit the one-shot kernel, and the pipelined kernel's
        // cross-GPU publish would go unchecked
        const size_t os_keep = w.oneshot_max;
        w.oneshot_max = 0;
        for (int i = 0; i < 2 && !rc; ++i) {
            const int k = calls++;
            const size_t c = ((size_t)1 << 20) / (size_t)n - 4 * (size_t)i;
            fill(sb, c, k, me);
            if (!rc) rc = allgather_node(sb, rb, c * 4, nullptr);
            check(rb, c * n, k, 2, (int)c, 0, "pipelined allgather");
        }
        w.oneshot_max = os_keep;
        // one-shot allgather and broadcast (k_oneshot_mv): a 12-byte block (byte by byte) and 16-byte
        // blocks, and a broadcast with a tail
        const size_t os_ag[2] = {3, 4096}, os_bc[2] = {3, 16387};
        for (int i = 0; i < 2 && !rc; ++i) {
            const int k = calls++;
            fill(sb, os_ag[i], k, me);
            if (!rc) rc = allgather_node(sb, rb, os_ag[i] * 4, nullptr);
            check(rb, os_ag[i] * n, k, 2, (int)os_ag[i], 0, "one-shot allgather");
        }
        for (int i = 0; i < 2 && !rc; ++i) {
            const int k = calls++;
            const int root = i == 0 ? n - 1 : 0;
            if (me == root) fill(rb, os_bc[i], k, root);
            else if (!rc) rc = hipMemsetAsync(rb, 0x5A, os_bc[i] * 4, st) == hipSuccess ? 0 : E_INTERN;
            if (!rc) rc = bcast_node(rb, os_bc[i] * 4, root, nullptr);
            check(rb, os_bc[i], k, 1, root, 0, "one-shot broadcast");
        }
        w.oneshot_max = 0;
        for (int i = 0; i < 2 && !rc; ++i) {
            const int k = calls++;
            const int root = i == 0 ? 0 : n - 1;
            const size_t c = ((size_t)1 << 18) + 3 * (size_t)i;
            if (me == root) fill(rb, c, k, root);
            else if (!rc) rc = hipMemsetAsync(rb, 0xA5, c * 4, st) == hipSuccess ? 0 : E_INTERN;
            if (!rc) rc = bcast_node(rb, c * 4, root, nullptr);
            check(rb, c, k, 1, root, 0, "pipelined broadcast");
        }
        w.oneshot_max = os_keep;
        // graph lane: a captured one-shot and a captured pipelined allreduce, replayed
        if (w.graph_lane && !rc) {
            hipStream_t cs = nullptr;
            const size_t gc[2] = {4096, (((size_t)1 << 20) / (16 * (size_t)n)) * 16 * (size_t)n};
            for (int g = 0; g < 2; ++g) fits(sb + (size_t)g * kGraphOff, gc[g]), fits(rb + (size_t)g * kGraphOff, gc[g]);
            hipGraph_t graph[2] = {};
            hipGraphExec_t ex[2] = {};
            if (hipStreamCreate(&cs) != hipSuccess) rc = E_INTERN;
            for (int g = 0; g < 2 && !rc; ++g) {
                if (hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) != hipSuccess) {
                    rc = E_INTERN;
                    break;
                }
                int crc;
                {
                    EnqueueScope q(true);
                    crc = ::allreduce_entry(sb + (size_t)g * kGraphOff, rb + (size_t)g * kGraphOff, gc[g], MPI_INT_H, MPI_SUM_H, cs);
                }
                if (hipStreamEndCapture(cs, &graph[g]) != hipSuccess || crc ||
                    hipGraphInstantiate(&ex[g], graph[g], nullptr, nullptr, 0) != hipSuccess)
                    rc = crc ? crc : E_INTERN;
            }
            hipStreamSynchronize(st);  // the blocking calls above are done before the replays
            for (int rep = 0; rep < 3 && !rc; ++rep)
                for (int g = 0; g < 2 && !rc; ++g) {
                    const int k = calls++;
                    if (!fits(sb + (size_t)g * kGraphOff, gc[g]) ||
                        (rc = launch_selftest_fill(sb + (size_t)g * kGraphOff, gc[g], seed_of(k), me, cs)))
                        break;
                    if (hipGraphLaunch(ex[g], cs) != hipSuccess) rc = E_INTERN;
                    if (!rc) rc = launch_selftest_check(rb + (size_t)g * kGraphOff, gc[g], seed_of(k), n, 0, 0, 0, bad + k, cs);
                    what[k] = "graph-lane allreduce";
                }
            if (cs && hipStreamSynchronize(cs) != hipSuccess) rc = rc ? rc : E_INTERN;
            if (!rc && check_err_word()) rc = E_OTHER;
            for (int g = 0; g < 2; ++g) {
                if (ex[g]) hipGraphExecDestroy(ex[g]);
                if (graph[g]) hipGraphDestroy(graph[g]);
            }
            if (cs) hipStreamDestroy(cs);
        }
        uint32_t hb[kMaxCalls] = {};
        if (hipStreamSynchronize(st) != hipSuccess || hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost) != hipSuccess)
            rc = rc ? rc : E_INTERN;
        int ok = rc == 0;
        for (int k = 0; k < calls && ok; ++k)
            if (hb[k]) {
                MV2_ERR("self-test (%s release): call %d (%s) returned %u wrong elements",
                        w.light_release ? "light" : "full", k, what[k] ? what[k] : "?", hb[k]);
                ok = 0;
            }
        if (rc) MV2_ERR("self-test: a call failed (MPI error class %d)", rc);
        // 1 = every element right, 0 = wrong elements, -1 = a call or launch failed; the retry below
        // is decided from these agreed values, never from this rank's own rc (a rank that stopped
        // while its peers ran the set again would leave them waiting for it)
        w.shm->r[me].selftest_ok = rc ? -1 : ok;
        host_barrier();
        int all_ok = 1, any_err = 0;
        for (int j = 0; j < n; ++j) {
            all_ok &= w.shm->r[j].selftest_ok == 1;
            any_err |= w.shm->r[j].selftest_ok < 0;
        }
        host_barrier();  // every rank has read every verdict
        if (all_ok) {
            verdict = 0;
            MV2_DEBUG("self-test passed: %d calls (light_release=%d)", calls, w.light_release);
            break;
        }
        verdict = E_INTERN;
        if (w.light_release && !any_err) {
            if (me == 0)
                fprintf(stderr, "[mv2amd] warning: device collective self-test failed with the light release; "
                                "using the full system-scope release\n");
            w.light_release = 0;
        } else {
            break;
        }
    }
    w.selftest_calls = calls;
    hipFree(sb);
    hipFree(rb);
    hipFree(bad);
    if (verdict) MV2_ERR("device collective self-test failed at MPI_Init (ranks %d): cross-GPU protocol broken", n);
    return verdict;
}

}  // namespace mv2
