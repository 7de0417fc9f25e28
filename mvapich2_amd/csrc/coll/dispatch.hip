// dispatch.hip — route (op, kind) to the per-group instantiations and hold
// the op-independent data-movement pipeline (all-gather / broadcast).
#include "kernels.h"
#include "pipe.h"

#include "../common.h"

namespace mv2 {

#define MV2_GROUPS(X) X(int8) X(int16) X(int32) X(int64) X(fp) X(cplx) X(pair)

#define MV2_DECL(g)                                                                                  \
    int grp_reduce_local_##g(int, int, const void *, void *, size_t, const LaunchCfg &);             \
    int grp_reduce_n_##g(int, int, const void *const *, int, void *, size_t, const TreeParams &,     \
                         const LaunchCfg &);                                                         \
    int grp_oneshot_##g(int, int, const OneShotArgs &, const LaunchCfg &);                           \
    int grp_pipe_##g(int, int, const PipeArgs &, const LaunchCfg &);                                 \
    int grp_touch_##g(hipStream_t);
MV2_GROUPS(MV2_DECL)
#undef MV2_DECL

// first group that recognises the kind wins (-1 = kind not in group)
#define MV2_TRY(g, fn, ...)                         \
    {                                               \
        int rc = grp_##fn##_##g(__VA_ARGS__);       \
        if (rc != -1) return rc;                    \
    }

int launch_reduce_local(int op, int kind, const void *in, void *inout, size_t count, size_t,
                        const LaunchCfg &cfg) {
#define X(g) MV2_TRY(g, reduce_local, op, kind, in, inout, count, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

int launch_reduce_n(int op, int kind, const void *const *srcs, int n, void *dst, size_t count, size_t,
                    const TreeParams &tp, const LaunchCfg &cfg) {
    if (n < 1 || n > kMaxRanks) return E_ARG;
#define X(g) MV2_TRY(g, reduce_n, op, kind, srcs, n, dst, count, tp, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

int launch_oneshot(int op, int kind, const OneShotArgs &a, size_t, const LaunchCfg &cfg) {
#define X(g) MV2_TRY(g, oneshot, op, kind, a, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

int launch_pipe_reduce(int op, int kind, const PipeArgs &a, const LaunchCfg &cfg) {
#define X(g) MV2_TRY(g, pipe, op, kind, a, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

int launch_pipe_copy(const PipeArgs &a, const LaunchCfg &cfg) {
    hipLaunchKernelGGL((k_pipe<NoReduce>), dim3(cfg.grid), dim3(kPipeThreads), 0, cfg.stream, a);
    return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
}

// ---------------------------------------------------------------------------
// One-shot allgather / broadcast (messages up to the one-shot limit): the pipelined kernel's two
// flag exchanges per round cost ~4 us more than the one-shot allreduce's one (osu 8 B at 2 shared
// ranks: allgather 15.8, bcast 15.0 against allreduce 11.2 us, profiles/r05c).  Workgroup b pushes
// partition b of the block this rank contributes (allgather: its own block; broadcast: the root's
// buffer, at the root only) into slot [me] of every peer's one-shot arena (this call's half), every
// rank raises its flag -- the non-roots of a broadcast too, so that no rank can reach call i + 2
// while a peer still reads call i's half (the one-shot allreduce's argument) -- waits for its
// peers' flags of workgroup b, and copies partition b of the slots it needs out of its own arena.
// Allgather blocks of 16-byte multiples move as vectors; a small block of any other size moves
// byte by byte through workgroup 0 (nvec = 0), as does a broadcast's tail.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_oneshot_mv(OneShotArgs a) {
    const int blk = blockIdx.x, G = gridDim.x;
    const size_t per = (a.nvec + G - 1) / G;
    const size_t vb = (size_t)blk * per < a.nvec ? (size_t)blk * per : a.nvec;
    const size_t ve = vb + per < a.nvec ? vb + per : a.nvec;
    const bool bc = a.mv == 2;
    const size_t tail0 = a.nvec * 16;
    uint64_t epoch = a.epoch;
    size_t poff = 0;
    if (a.dseq) {  // graph lane: this replay's epoch and arena half
        const SeqBase q = dseq_read(a.dseq);
        epoch = q.epoch + 1;
        poff = (q.os & 1) * a.half;
    }
    const size_t myslot = poff + (size_t)a.me * a.slot_bytes;
    if (!bc || a.me == a.root) {
        const v4u *src = (const v4u *)a.send;
        for (size_t i = vb + threadIdx.x; i < ve; i += kThreads) {
            const v4u x = src[i];
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j)
                if (j < a.n && j != a.me) ((v4u *)(a.arena_peer.p[j] + myslot))[i] = x;
            if (!bc && a.send != a.recv + (size_t)a.me * a.pitch) ((v4u *)(a.recv + (size_t)a.me * a.pitch))[i] = x;
        }
        if (blk == 0)
            for (size_t e = tail0 + threadIdx.x; e < a.count; e += kThreads) {
                const char c = a.send[e];
#pragma unroll
                for (int j = 0; j < kMaxRanks; ++j)
                    if (j < a.n && j != a.me) a.arena_peer.p[j][myslot + e] = c;
                if (!bc && a.send != a.recv + (size_t)a.me * a.pitch) a.recv[(size_t)a.me * a.pitch + e] = c;
            }
    }
    signal_peers(a.sig_peer, a.n, a.me, blk, epoch, a.light != 0);
    if (wait_peers(a.sig_own, a.n, blk, epoch, a.err, a.timeout, a.light != 0)) {
        for (int j = 0; j < a.n; ++j) {
            if (j == a.me || (bc && j != a.root)) continue;
            const char *slot = a.arena_own + poff + (size_t)j * a.slot_bytes;
            char *dst = bc ? a.recv : a.recv + (size_t)j * a.pitch;
            for (size_t i = vb + threadIdx.x; i < ve; i += kThreads) ((v4u *)dst)[i] = ld_nt((const v4u *)slot + i);
            if (blk == 0)
                for (size_t e = tail0 + threadIdx.x; e < a.count; e += kThreads)
                    dst[e] = __builtin_nontemporal_load(slot + e);
        }
    }
    if (a.dseq) dseq_advance(a.dseq, 1, 0, 1);
    block_done(a.done);
}

int launch_oneshot_mv(const OneShotArgs &a, const LaunchCfg &cfg) {
    static const int cap = resident_grid((const void *)k_oneshot_mv, cfg);
    const int g = cfg.grid < cap ? cfg.grid : cap;
    hipLaunchKernelGGL(k_oneshot_mv, dim3(g), dim3(kThreads), 0, cfg.stream, a);
    return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
}

// ---------------------------------------------------------------------------
// Code-object loading.  HIP loads a translation unit's gfx950 code object at the first launch of
// one of its kernels; MPI_Init launches one empty kernel per unit so that the load happens (and
// is timed) there rather than inside an application's first call of each type group.
// ---------------------------------------------------------------------------
__global__ void k_touch_dispatch() {}
int launch_pack_touch(hipStream_t st);  // pack/pack.hip

int launch_touch_all(hipStream_t st) {
    hipLaunchKernelGGL(k_touch_dispatch, dim3(1), dim3(64), 0, st);
    if (hipGetLastError() != hipSuccess) return E_INTERN;
#define X(g) \
    if (grp_touch_##g(st)) return E_INTERN;
    MV2_GROUPS(X)
#undef X
    return launch_pack_touch(st);
}

// ---------------------------------------------------------------------------
// MPI_Init self-test operands (runtime/coll.cpp coll_selftest): rank r's element i of call
// `seed` is st_hash(seed, r, i); the check recomputes what every element of a result must be
// and counts the elements that differ (integer arithmetic mod 2^32: any reduction order agrees).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t st_hash(uint32_t seed, uint32_t r, uint64_t i) {
    uint32_t x = (uint32_t)i * 0x9E3779B1u ^ (uint32_t)(i >> 32) ^ seed ^ (r + 1u) * 0x85EBCA77u;
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(kThreads) void k_st_fill(uint32_t *p, size_t n, uint32_t seed, int rank) {
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kThreads)
        p[i] = st_hash(seed, (uint32_t)rank, i);
}

// mode 0: element i = sum over ranks of st_hash(seed, r, base + i)   (allreduce, reduce-scatter block)
// mode 1: element i = st_hash(seed, arg, base + i)                  (broadcast from rank arg)
// mode 2: element i = st_hash(seed, i / arg, i % arg)               (allgather of arg elements per rank)
__global__ __launch_bounds__(kThreads) void k_st_check(const uint32_t *p, size_t n, uint32_t seed, int nranks,
                                                       int mode, int arg, uint64_t base, uint32_t *bad) {
    uint32_t nb = 0;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kThreads) {
        uint32_t want = 0;
        if (mode == 0) {
            for (int r = 0; r < nranks; ++r) want += st_hash(seed, (uint32_t)r, base + i);
        } else if (mode == 1) {
            want = st_hash(seed, (uint32_t)arg, base + i);
        } else {
            want = st_hash(seed, (uint32_t)(i / (size_t)arg), i % (size_t)arg);
        }
        nb += p[i] != want ? 1u : 0u;
    }
    if (nb) atomicAdd(bad, nb);
}

static unsigned st_grid(size_t n) {
    const size_t g = (n + kThreads - 1) / kThreads;
    return (unsigned)(g < 1 ? 1 : (g > 1024 ? 1024 : g));
}

int launch_selftest_fill(uint32_t *p, size_t n, uint32_t seed, int rank, hipStream_t st) {
    hipLaunchKernelGGL(k_st_fill, dim3(st_grid(n)), dim3(kThreads), 0, st, p, n, seed, rank);
    return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
}

int launch_selftest_check(const uint32_t *p, size_t n, uint32_t seed, int nranks, int mode, int arg, uint64_t base,
                          uint32_t *bad, hipStream_t st) {
    hipLaunchKernelGGL(k_st_check, dim3(st_grid(n)), dim3(kThreads), 0, st, p, n, seed, nranks, mode, arg, base, bad);
    return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
}

}  // namespace mv2
