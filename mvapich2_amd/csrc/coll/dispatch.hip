// dispatch.hip — route (op, kind) to the per-group instantiations and hold
// the op-independent data-movement kernels (all-gather / broadcast reads).
#include "kernels.h"

#include "../common.h"

namespace mv2 {

#define MV2_GROUPS(X) X(int8) X(int16) X(int32) X(int64) X(fp) X(cplx) X(pair)

#define MV2_DECL(g)                                                                                  \
    int grp_reduce_local_##g(int, int, const void *, void *, size_t, const LaunchCfg &);             \
    int grp_reduce_n_##g(int, int, const void *const *, int, void *, size_t, const TreeParams &,     \
                         const LaunchCfg &);                                                         \
    int grp_oneshot_##g(int, int, const OneShotArgs &, const LaunchCfg &);                           \
    int grp_twoshot_##g(int, int, const TwoShotArgs &, const LaunchCfg &);                           \
    int grp_rs_##g(int, int, const RsArgs &, const LaunchCfg &);
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

int launch_twoshot(int op, int kind, const TwoShotArgs &a, size_t, const LaunchCfg &cfg) {
#define X(g) MV2_TRY(g, twoshot, op, kind, a, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

int launch_rs(int op, int kind, const RsArgs &a, size_t, const LaunchCfg &cfg) {
#define X(g) MV2_TRY(g, rs, op, kind, a, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

// ---------------------------------------------------------------------------
// Gather-read kernel: dst[dst_off[j] .. + bytes) = src[j][0 .. bytes) for every
// rank j with src[j] != nullptr (all-gather: every j; broadcast: the root).
// E0 entry barrier (sources ready), E1 exit barrier (peers done reading).
// Vector path when every address is 16-byte aligned and bytes % 16 == 0.
// ---------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(kThreads) void k_gather(GatherArgs a, int vec) {
    const int blk = blockIdx.x, G = gridDim.x;
    signal_peers(a.sig_peer, a.n, a.me, blk, a.epoch);
    if (!wait_peers(a.sig_own, a.n, blk, a.epoch, a.err, a.timeout)) return;
    if (vec) {
        const size_t nv = a.bytes / 16;
        const size_t stride = (size_t)G * kThreads * U;
        for (size_t base = (size_t)blk * kThreads * U + threadIdx.x; base < nv; base += stride) {
            v4u v[U][kMaxRanks];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t i = base + (size_t)u * kThreads;
#pragma unroll
                for (int j = 0; j < kMaxRanks; ++j)
                    v[u][j] = (j < a.n && a.src.p[j] && i < nv) ? ld_nt((const v4u *)a.src.p[j] + i) : v4u{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t i = base + (size_t)u * kThreads;
#pragma unroll
                for (int j = 0; j < kMaxRanks; ++j)
                    if (j < a.n && a.src.p[j] && i < nv) st_nt((v4u *)(a.dst + a.dst_off[j]) + i, v[u][j]);
            }
        }
    } else {
        const size_t stride = (size_t)G * kThreads;
        for (size_t i = (size_t)blk * kThreads + threadIdx.x; i < a.bytes; i += stride) {
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j)
                if (j < a.n && a.src.p[j]) (a.dst + a.dst_off[j])[i] = a.src.p[j][i];
        }
    }
    signal_peers(a.sig_peer, a.n, a.me, blk, a.epoch + 1);
    wait_peers(a.sig_own, a.n, blk, a.epoch + 1, a.err, a.timeout);
}

int launch_gather(const GatherArgs &a, const LaunchCfg &cfg) {
    bool vec = a.bytes % 16 == 0 && (uintptr_t)a.dst % 16 == 0;
    for (int j = 0; j < a.n; ++j) {
        if (!a.src.p[j]) continue;
        vec = vec && ((uintptr_t)a.src.p[j] % 16 == 0) && (a.dst_off[j] % 16 == 0);
    }
    static const int cap = resident_grid((const void *)k_gather<2>, cfg);
    const int g = cfg.grid < cap ? cfg.grid : cap;
    hipLaunchKernelGGL((k_gather<2>), dim3(g), dim3(kThreads), 0, cfg.stream, a, vec ? 1 : 0);
    return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
}

}  // namespace mv2
