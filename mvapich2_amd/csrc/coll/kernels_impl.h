// kernels_impl.h — templated gfx950 kernels for the MPI_Op layer and the
// device collectives.  Instantiated per (op, kind) in kernels_*.hip.
//
// Data layout: every buffer is addressed as 16-byte vectors (v4u) holding
// 16/sizeof(T) elements (pair records with padding keep the accumulator's
// padding bytes); elements past the last whole vector are a scalar tail.
// All kernels are HBM- or xGMI-bound: 256-thread workgroups, U vectors per
// thread in flight per source, grid-stride over tiles, non-temporal stores
// for results that are not re-read by the kernel.
#pragma once
#include <hip/hip_runtime.h>

#include "../ops/functors.h"
#include "kernels.h"

namespace mv2 {

// ============================================================================
// MPI_Reduce_local: inout[i] = op(inout[i], in[i])   (reduce_local.c:139)
// ============================================================================
// Streamed shape chosen by tools/rl_variants.hip on MI355X (random fp32
// operands, 256 MiB): non-temporal loads + plain stores, 512 threads x 2
// vectors per thread, one tile per workgroup (full grid): 6.7 TB/s, against
// 6.25 TB/s for non-temporal stores on a 4096-workgroup grid-stride grid.
constexpr int kRLThreads = 512;
template <class Rd, int U>
__global__ __launch_bounds__(kRLThreads) void k_reduce_local(const v4u *__restrict__ in,
                                                             v4u *__restrict__ io, size_t nvec,
                                                             const typename Rd::T *__restrict__ tin,
                                                             typename Rd::T *__restrict__ tio,
                                                             size_t tail_beg, size_t tail_end, Done dn) {
    const size_t stride = (size_t)gridDim.x * kRLThreads * U;
    for (size_t base = (size_t)blockIdx.x * kRLThreads * U + threadIdx.x; base < nvec; base += stride) {
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * kRLThreads;
            if (i < nvec) {
                a[u] = ld_nt(&io[i]);
                b[u] = ld_nt(&in[i]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * kRLThreads;
            if (i < nvec) io[i] = vapply<Rd>(a[u], b[u]);
        }
    }
    if (blockIdx.x == 0)
        for (size_t e = tail_beg + threadIdx.x; e < tail_end; e += kRLThreads) tio[e] = Rd::apply(tio[e], tin[e]);
    block_done(dn);
}

// element-granular variant for buffers that are not 16-byte aligned
template <class Rd>
__global__ __launch_bounds__(kThreads) void k_reduce_local_elem(const typename Rd::T *__restrict__ in,
                                                                typename Rd::T *__restrict__ io,
                                                                size_t count, Done dn) {
    const size_t stride = (size_t)gridDim.x * kThreads;
    for (size_t e = (size_t)blockIdx.x * kThreads + threadIdx.x; e < count; e += stride)
        io[e] = Rd::apply(io[e], in[e]);
    block_done(dn);
}

// small operands (the metric's 8-byte call): one wave, element by element, then lane 0 raises the
// completion word with a system-scope release (block_done's one-workgroup path).  Against the
// 512-thread streaming kernel this dispatches one wave instead of eight and passes 32 bytes of
// arguments instead of 88 (the host launch and the CP's dispatch are most of an 8-byte call:
// tools/diag/rl_lat.cpp, profiles/r06e)
template <class Rd>
__global__ __launch_bounds__(64) void k_reduce_local_tiny(const typename Rd::T *__restrict__ in,
                                                          typename Rd::T *__restrict__ io, uint32_t count,
                                                          uint64_t *flag, uint64_t seq) {
    // every argument in SGPRs before the first branch: the kernel-argument fetches issue together
    // and are waited for once (left to the compiler, the count, the operand pointers and the word's
    // pointer and value are three dependent fetches from host memory, ~0.1 us each)
    asm volatile("" ::"s"(in), "s"(io), "s"(count), "s"(flag), "s"(seq));
    for (uint32_t e = threadIdx.x; e < count; e += 64) io[e] = Rd::apply(io[e], in[e]);
    // One wave: the release's own `buffer_wbl2; s_waitcnt vmcnt(0)` (issued after the store
    // instruction that wrote every lane's element) covers all 64 lanes' stores, so no separate wait
    // for them first -- that wait made the stores' acknowledgement and the write-back two round
    // trips (0.2-0.3 us of the 8-byte call, profiles/r06/r06w-r06y)
    if (flag && threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int OP, int K>
struct LReduceLocal {
    static int run(const void *in, void *inout, size_t count, const LaunchCfg &cfg) {
        using Rd = R<OP, K>;
        using T = typename Rd::T;
        constexpr size_t VPT = 16 / sizeof(T);
        if (count * sizeof(T) <= cfg.tiny_max && count <= 0xffffffffu) {
            hipLaunchKernelGGL((k_reduce_local_tiny<Rd>), dim3(1), dim3(64), 0, cfg.stream, (const T *)in, (T *)inout,
                               (uint32_t)count, cfg.done.flag, cfg.done.seq);
            return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
        }
        const bool aligned = ((uintptr_t)in % 16 == 0) && ((uintptr_t)inout % 16 == 0);
        if (!aligned) {
            size_t g = (count + kThreads - 1) / kThreads;
            if (g > (size_t)cfg.grid) g = cfg.grid;
            if (g == 0) g = 1;
            hipLaunchKernelGGL((k_reduce_local_elem<Rd>), dim3(g), dim3(kThreads), 0, cfg.stream,
                               (const T *)in, (T *)inout, count, cfg.done);
            return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
        }
        const size_t nvec = count / VPT;
        const size_t tile = (size_t)kRLThreads * 2;
        size_t g = (nvec + tile - 1) / tile;
        if (g > (size_t)cfg.grid) g = cfg.grid;
        if (g == 0) g = 1;
        hipLaunchKernelGGL((k_reduce_local<Rd, 2>), dim3(g), dim3(kRLThreads), 0, cfg.stream,
                           (const v4u *)in, (v4u *)inout, nvec, (const T *)in, (T *)inout,
                           nvec * VPT, count, cfg.done);
        return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
    }
};

// ============================================================================
// n-input reduction helpers (sources may be peer-mapped pointers)
// ============================================================================
template <class Rd>
__device__ __forceinline__ int elem_owner(const TreeParams &tp, size_t e) {
    if (tp.owner_fixed >= 0) return tp.owner_fixed;
    size_t b = tp.rs_blk ? e / tp.rs_blk : 0;
    if (b > (size_t)(tp.pof2 - 1)) b = tp.pof2 - 1;
    return brev_bits((int)b, tp.lg);
}

// reduce n 16-byte vectors (v[j] from rank j) whose first element index is e0.
// Program order (linear == 4): fixed_blk >= 0 is the program block of the
// whole vector when the caller knows it (hoisted out of the loop).
template <class Rd, int ORD = -1>
__device__ __forceinline__ v4u vreduce_n(const v4u (&v)[kMaxRanks], int n, const TreeParams &tp,
                                         size_t e0, int fixed_blk = -1) {
    using T = typename Rd::T;
    constexpr int N = 16 / sizeof(T);
    T t[kMaxRanks][N];
#pragma unroll
    for (int j = 0; j < kMaxRanks; ++j) __builtin_memcpy(t[j], &v[j], 16);
    T out[N];
    const int lin = ORD >= 0 ? ORD : tp.linear;
    if constexpr (ORD == 4) {  // callers dispatch program order explicitly (no copy of tp.ps)
        const ProgSet &ps = tp.ps;
        const int b0 = fixed_blk >= 0 ? fixed_blk : prog_block(ps, e0);
        const int bN = fixed_blk >= 0 ? fixed_blk : prog_block(ps, e0 + N - 1);
#pragma unroll
        for (int i = 0; i < N; ++i) {
            T col[kMaxRanks];
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j) col[j] = t[j][i];
            const int b = (b0 == bN) ? b0 : prog_block(ps, e0 + i);
            out[i] = prog_eval<Rd>(col, ps.p[b]);
        }
        v4u r;
        __builtin_memcpy(&r, out, 16);
        return r;
    } else {
        const int own0 = lin ? 0 : elem_owner<Rd>(tp, e0);
        const int ownN = lin ? 0 : elem_owner<Rd>(tp, e0 + N - 1);
#pragma unroll
        for (int i = 0; i < N; ++i) {
            T col[kMaxRanks];
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j) col[j] = t[j][i];
            const int own = (own0 == ownN) ? own0 : elem_owner<Rd>(tp, e0 + i);
            out[i] = tree_reduce<Rd, ORD>(col, n, tp.linear, tp.pof2, tp.rem, own);
        }
        v4u r;
        __builtin_memcpy(&r, out, 16);
        return r;
    }
}

// one element's reduction in the call's order (scalar tails)
template <class Rd>
__device__ __forceinline__ typename Rd::T col_reduce(const typename Rd::T (&col)[kMaxRanks], int n,
                                                     const TreeParams &tp, size_t e) {
    if (tp.linear == 4) return prog_eval<Rd>(col, tp.ps.p[prog_block(tp.ps, e)]);
    return tree_reduce<Rd>(col, n, tp.linear, tp.pof2, tp.rem, elem_owner<Rd>(tp, e));
}

template <class Rd>
__device__ __forceinline__ typename Rd::T sreduce_n(const typename Rd::T *const *src, int n,
                                                    const TreeParams &tp, size_t e) {
    using T = typename Rd::T;
    T col[kMaxRanks];
#pragma unroll
    for (int j = 0; j < kMaxRanks; ++j) col[j] = (j < n) ? src[j][e] : src[0][e];
    return col_reduce<Rd>(col, n, tp, e);
}

// plain n-source reduction into dst (single process; used by mv2h_reduce_n and tests)
template <class Rd, int U>
__global__ __launch_bounds__(kThreads) void k_reduce_n(PeerTable src, int n, char *dst, size_t count,
                                                       size_t nvec, TreeParams tp) {
    using T = typename Rd::T;
    constexpr int N = 16 / sizeof(T);
    const size_t stride = (size_t)gridDim.x * kThreads * U;
    for (size_t base = (size_t)blockIdx.x * kThreads * U + threadIdx.x; base < nvec; base += stride) {
        v4u v[U][kMaxRanks];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * kThreads;
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j)
                v[u][j] = (j < n && i < nvec) ? ld_nt((const v4u *)src.p[j] + i) : v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * kThreads;
            if (i < nvec)
                ((v4u *)dst)[i] = tp.linear == 4 ? vreduce_n<Rd, 4>(v[u], n, tp, i * N) : vreduce_n<Rd>(v[u], n, tp, i * N);
        }
    }
    if (blockIdx.x == 0) {
        const T *s[kMaxRanks];
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j) s[j] = (const T *)src.p[j];
        for (size_t e = nvec * N + threadIdx.x; e < count; e += kThreads) ((T *)dst)[e] = sreduce_n<Rd>(s, n, tp, e);
    }
}

template <class Rd>
__global__ __launch_bounds__(kThreads) void k_reduce_n_elem(PeerTable src, int n, char *dst, size_t count,
                                                            TreeParams tp) {
    using T = typename Rd::T;
    const T *s[kMaxRanks];
#pragma unroll
    for (int j = 0; j < kMaxRanks; ++j) s[j] = (const T *)src.p[j];
    const size_t stride = (size_t)gridDim.x * kThreads;
    for (size_t e = (size_t)blockIdx.x * kThreads + threadIdx.x; e < count; e += stride)
        ((T *)dst)[e] = sreduce_n<Rd>(s, n, tp, e);
}

template <int OP, int K>
struct LReduceN {
    static int run(const void *const *srcs, int n, void *dst, size_t count, const TreeParams &tp,
                   const LaunchCfg &cfg) {
        using Rd = R<OP, K>;
        using T = typename Rd::T;
        constexpr size_t VPT = 16 / sizeof(T);
        PeerTable pt{};
        bool aligned = (uintptr_t)dst % 16 == 0;
        for (int j = 0; j < n; ++j) {
            pt.p[j] = (const char *)srcs[j];
            aligned = aligned && ((uintptr_t)srcs[j] % 16 == 0);
        }
        for (int j = n; j < kMaxRanks; ++j) pt.p[j] = pt.p[0];
        if (!aligned) {
            size_t g = (count + kThreads - 1) / kThreads;
            if (g > (size_t)cfg.grid) g = cfg.grid;
            if (g == 0) g = 1;
            hipLaunchKernelGGL((k_reduce_n_elem<Rd>), dim3(g), dim3(kThreads), 0, cfg.stream, pt, n,
                               (char *)dst, count, tp);
        } else {
            // one vector per thread in flight: the n-source reduction serves the order tests and
            // the leaders' steps across nodes (host-staged, link-bound), so its code stays small
            const size_t nvec = count / VPT;
            size_t g = (nvec + kThreads - 1) / kThreads;
            if (g > (size_t)cfg.grid) g = cfg.grid;
            if (g == 0) g = 1;
            hipLaunchKernelGGL((k_reduce_n<Rd, 1>), dim3(g), dim3(kThreads), 0, cfg.stream, pt, n,
                               (char *)dst, count, nvec, tp);
        }
        return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
    }
};

// ============================================================================
// One-shot allreduce (small messages): push my sendbuf into every peer's
// arena slot, flag, then reduce all n slots locally in reference order.
// No exit barrier: the arena half used alternates per call (parity), and a
// peer can only reach call i+2 after every rank finished call i.
// ============================================================================
// Graph lane (DevSeq, kernels.h): every workgroup reads the call's base when it starts; the
// last workgroup to finish advances it, after all of them have read it.
struct SeqBase {
    uint64_t epoch, round, os;
};
__device__ __forceinline__ SeqBase dseq_read(DevSeq *d) {
    __shared__ uint64_t s_q[3];
    if (threadIdx.x == 0) {
        s_q[0] = __hip_atomic_load(&d->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_q[1] = __hip_atomic_load(&d->round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_q[2] = __hip_atomic_load(&d->os, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return SeqBase{s_q[0], s_q[1], s_q[2]};
}
__device__ __forceinline__ void dseq_advance(DevSeq *d, uint64_t de, uint64_t dr, uint64_t dos) {
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(&d->arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1u == gridDim.x) {
        __hip_atomic_store(&d->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (de) __hip_atomic_fetch_add(&d->epoch, de, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (dr) __hip_atomic_fetch_add(&d->round, dr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (dos) __hip_atomic_fetch_add(&d->os, dos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
}

// SMALL: an operand with no whole 16-byte vectors (nvec == 0), element by element in workgroup 0;
// the vector phases are compiled out, so the kernel's code is a fraction of the general body's
// (the 8-byte allreduce: 45 KB of code against the one-shot allgather's 4.7 KB, profiles/r05ay)
template <class Rd, bool PROG, bool SMALL = false>
__device__ __forceinline__ void oneshot_body(const OneShotArgs &a, uint64_t epoch, size_t poff) {
    using T = typename Rd::T;
    constexpr int N = 16 / sizeof(T);
    const int blk = blockIdx.x, G = gridDim.x;
    const size_t nvec = SMALL ? 0 : a.nvec;
    const size_t per = (nvec + G - 1) / G;
    const size_t vb = (size_t)blk * per;
    const size_t ve = vb + per < nvec ? vb + per : nvec;
    const v4u *send = (const v4u *)a.send;
    // phase A: push my data to every peer's slot (me)
    if constexpr (!SMALL)
    for (size_t i = vb + threadIdx.x; i < ve; i += kThreads) {
        const v4u x = send[i];
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j)
            if (j < a.n && j != a.me) ((v4u *)(a.arena_peer.p[j] + poff + (size_t)a.me * a.slot_bytes))[i] = x;
    }
    const size_t tail0 = nvec * N;
    if (blk == 0) {
        for (size_t e = tail0 + threadIdx.x; e < a.count; e += kThreads) {
            const T x = ((const T *)a.send)[e];
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j)
                if (j < a.n && j != a.me) ((T *)(a.arena_peer.p[j] + poff + (size_t)a.me * a.slot_bytes))[e] = x;
        }
    }
    signal_peers(a.sig_peer, a.n, a.me, blk, epoch, a.light != 0);
    if (!wait_peers(a.sig_own, a.n, blk, epoch, a.err, a.timeout, a.light != 0)) return;
    const char *arena_own = a.arena_own + poff;
    // phase B: reduce the n slots (own data straight from sendbuf; arena slots with
    // non-temporal loads, which the light acquire relies on)
    auto load = [&](size_t i, v4u (&v)[kMaxRanks]) {
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j)
            v[j] = (j >= a.n) ? v4u{0, 0, 0, 0} : (j == a.me) ? send[i] : ld_nt((const v4u *)(arena_own + (size_t)j * a.slot_bytes) + i);
    };
    if constexpr (SMALL) {
    } else if constexpr (PROG) {
        // program order: the block of a range that lies in one block is fixed once
        int fb = -1;
        if (ve > vb) {
            const int b0 = prog_block(a.tp.ps, vb * N), b1 = prog_block(a.tp.ps, ve * N - 1);
            if (b0 == b1) fb = b0;
        }
        for (size_t i = vb + threadIdx.x; i < ve; i += kThreads) {
            v4u v[kMaxRanks];
            load(i, v);
            ((v4u *)a.recv)[i] = vreduce_n<Rd, 4>(v, a.n, a.tp, i * N, fb);
        }
    } else {
        // a butterfly owner that is constant over this workgroup's range is fixed once (no
        // per-vector 64-bit division)
        TreeParams tp = a.tp;
        if (!tp.linear && tp.owner_fixed < 0 && ve > vb) {
            const int o0 = elem_owner<Rd>(tp, vb * N), o1 = elem_owner<Rd>(tp, ve * N - 1);
            if (o0 == o1) tp.owner_fixed = o0;
        }
        for (size_t i = vb + threadIdx.x; i < ve; i += kThreads) {
            v4u v[kMaxRanks];
            load(i, v);
            ((v4u *)a.recv)[i] = vreduce_n<Rd>(v, a.n, tp, i * N);
        }
    }
    if (blk == 0) {
        for (size_t e = tail0 + threadIdx.x; e < a.count; e += kThreads) {
            T col[kMaxRanks];
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j)
                col[j] = (j >= a.n || j == a.me) ? ((const T *)a.send)[e]
                                                 : ld_nt_elem((const T *)(arena_own + (size_t)j * a.slot_bytes) + e);
            if constexpr (PROG) ((T *)a.recv)[e] = prog_eval<Rd>(col, a.tp.ps.p[prog_block(a.tp.ps, e)]);
            else ((T *)a.recv)[e] = tree_reduce<Rd>(col, a.n, a.tp.linear, a.tp.pof2, a.tp.rem, elem_owner<Rd>(a.tp, e));
        }
    }
}

template <class Rd, bool PROG, bool SMALL = false>
__global__ __launch_bounds__(kThreads) void k_oneshot(OneShotArgs a) {
    uint64_t epoch = a.epoch;
    size_t poff = 0;
    if (a.dseq) {  // graph lane: this replay's epoch and arena half
        const SeqBase q = dseq_read(a.dseq);
        epoch = q.epoch + 1;
        poff = (q.os & 1) * a.half;
    }
    oneshot_body<Rd, PROG, SMALL>(a, epoch, poff);
    if (a.dseq) dseq_advance(a.dseq, 1, 0, 1);
    block_done(a.done);
}

// One-shot reduce-scatter (small messages): workgroup b pushes, to every peer j, partition b of
// j's block of my operand, flags, then reduces partition b of my own block from the n slots in
// program order — the flag it waits for covers exactly the vectors it reads.  Block tails
// (elements past the last whole vector) go through workgroup 0 on both sides.
// SMALL: nvec == 0 with the vector phases compiled out (the compact kernel, as k_oneshot's)
template <class Rd, bool SMALL = false>
__global__ __launch_bounds__(kThreads) void k_oneshot_rs(OneShotArgs a) {
    using T = typename Rd::T;
    constexpr int N = 16 / sizeof(T);
    const int blk = blockIdx.x, G = gridDim.x;
    uint64_t epoch = a.epoch;
    size_t poff = 0;
    if (a.dseq) {
        const SeqBase q = dseq_read(a.dseq);
        epoch = q.epoch + 1;
        poff = (q.os & 1) * a.half;
    }
    const v4u *send = (const v4u *)a.send;
    // nvec == 0: small blocks that do not start on 16-byte boundaries, element by element in
    // workgroup 0 (the vector range of every block is then empty)
    const bool sc = SMALL || a.nvec == 0;
    for (int j = 0; j < a.n; ++j) {
        if (j == a.me) continue;
        const size_t v0 = a.wlo[j] / N, v1 = sc ? v0 : (a.wlo[j] + a.wcnt[j]) / N;
        v4u *dst = (v4u *)(a.arena_peer.p[j] + poff + (size_t)a.me * a.slot_bytes);
        if constexpr (!SMALL) {
            const size_t per = (v1 - v0 + G - 1) / G;
            const size_t b0 = v0 + (size_t)blk * per, b1 = b0 + per < v1 ? b0 + per : v1;
            for (size_t i = b0 + threadIdx.x; i < b1; i += kThreads) dst[i] = send[i];
        }
        if (blk == 0)
            for (size_t e = (sc ? a.wlo[j] : v1 * N) + threadIdx.x; e < a.wlo[j] + a.wcnt[j]; e += kThreads)
                ((T *)dst)[e] = ((const T *)a.send)[e];
    }
    signal_peers(a.sig_peer, a.n, a.me, blk, epoch, a.light != 0);
    if (wait_peers(a.sig_own, a.n, blk, epoch, a.err, a.timeout, a.light != 0)) {
        const char *arena_own = a.arena_own + poff;
        const size_t lo = a.wlo[a.me], hi = lo + a.wcnt[a.me];
        const size_t v0 = lo / N, v1 = sc ? v0 : hi / N;
        if constexpr (!SMALL) {
            const size_t per = (v1 - v0 + G - 1) / G;
            const size_t b0 = v0 + (size_t)blk * per, b1 = b0 + per < v1 ? b0 + per : v1;
            int fb = -1;
            if (b1 > b0) {
                const int p0 = prog_block(a.tp.ps, b0 * N), p1 = prog_block(a.tp.ps, b1 * N - 1);
                if (p0 == p1) fb = p0;
            }
            for (size_t i = b0 + threadIdx.x; i < b1; i += kThreads) {
                v4u v[kMaxRanks];
#pragma unroll
                for (int j = 0; j < kMaxRanks; ++j)
                    v[j] = (j >= a.n) ? v4u{0, 0, 0, 0}
                                      : (j == a.me) ? send[i] : ld_nt((const v4u *)(arena_own + (size_t)j * a.slot_bytes) + i);
                ((v4u *)a.recv)[i - v0] = vreduce_n<Rd, 4>(v, a.n, a.tp, i * N, fb);
            }
        }
        if (blk == 0)
            for (size_t e = (sc ? lo : v1 * N) + threadIdx.x; e < hi; e += kThreads) {
                T col[kMaxRanks];
#pragma unroll
                for (int j = 0; j < kMaxRanks; ++j)
                    col[j] = (j >= a.n || j == a.me) ? ((const T *)a.send)[e]
                                                     : ld_nt_elem((const T *)(arena_own + (size_t)j * a.slot_bytes) + e);
                ((T *)a.recv)[e - lo] = prog_eval<Rd>(col, a.tp.ps.p[prog_block(a.tp.ps, e)]);
            }
    }
    if (a.dseq) dseq_advance(a.dseq, 1, 0, 1);
    block_done(a.done);
}

template <int OP, int K>
struct LOneShot {
    static int run(const OneShotArgs &a, const LaunchCfg &cfg) {
        using Rd = R<OP, K>;
        const bool prog = a.tp.linear == 4;
        if (a.rs) {
            if (!prog) return E_ARG;  // a reduce-scatter block is always evaluated in program order
            if (a.nvec == 0 && cfg.grid == 1) {
                hipLaunchKernelGGL((k_oneshot_rs<Rd, true>), dim3(1), dim3(kThreads), 0, cfg.stream, a);
                return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
            }
            static const int cap2 = resident_grid((const void *)k_oneshot_rs<Rd>, cfg);
            const int g = cfg.grid < cap2 ? cfg.grid : cap2;
            hipLaunchKernelGGL((k_oneshot_rs<Rd>), dim3(g), dim3(kThreads), 0, cfg.stream, a);
            return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
        }
        if (a.nvec == 0 && cfg.grid == 1) {  // no whole vector: the compact element-wise kernel
            if constexpr (Rd::kOrderFree) {
                hipLaunchKernelGGL((k_oneshot<Rd, false, true>), dim3(1), dim3(kThreads), 0, cfg.stream, a);
            } else {
                if (prog) hipLaunchKernelGGL((k_oneshot<Rd, true, true>), dim3(1), dim3(kThreads), 0, cfg.stream, a);
                else hipLaunchKernelGGL((k_oneshot<Rd, false, true>), dim3(1), dim3(kThreads), 0, cfg.stream, a);
            }
            return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
        }
        static const int cap0 = resident_grid((const void *)k_oneshot<Rd, false>, cfg);
        if constexpr (Rd::kOrderFree) {  // every order gives the same bits: the LINEAR body
            const int g = cfg.grid < cap0 ? cfg.grid : cap0;
            hipLaunchKernelGGL((k_oneshot<Rd, false>), dim3(g), dim3(kThreads), 0, cfg.stream, a);
        } else {
            static const int cap1 = resident_grid((const void *)k_oneshot<Rd, true>, cfg);
            const int cap = prog ? cap1 : cap0;
            const int g = cfg.grid < cap ? cfg.grid : cap;
            if (prog) hipLaunchKernelGGL((k_oneshot<Rd, true>), dim3(g), dim3(kThreads), 0, cfg.stream, a);
            else hipLaunchKernelGGL((k_oneshot<Rd, false>), dim3(g), dim3(kThreads), 0, cfg.stream, a);
        }
        return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
    }
};
// ---------------- runtime (op, kind) -> template dispatch ----------------
template <template <int, int> class L, int OP, int K, class... A>
inline int call_if(A &&...args) {
    if constexpr (legal<OP, K>()) return L<OP, canon_kind<OP, K>()>::run(static_cast<A &&>(args)...);
    else return E_OP;
}

template <template <int, int> class L, int K, class... A>
inline int dispatch_op(int op, A &&...args) {
    switch (op) {
    case OP_MAX: return call_if<L, OP_MAX, K>(static_cast<A &&>(args)...);
    case OP_MIN: return call_if<L, OP_MIN, K>(static_cast<A &&>(args)...);
    case OP_SUM: return call_if<L, OP_SUM, K>(static_cast<A &&>(args)...);
    case OP_PROD: return call_if<L, OP_PROD, K>(static_cast<A &&>(args)...);
    case OP_LAND: return call_if<L, OP_LAND, K>(static_cast<A &&>(args)...);
    case OP_BAND: return call_if<L, OP_BAND, K>(static_cast<A &&>(args)...);
    case OP_LOR: return call_if<L, OP_LOR, K>(static_cast<A &&>(args)...);
    case OP_BOR: return call_if<L, OP_BOR, K>(static_cast<A &&>(args)...);
    case OP_LXOR: return call_if<L, OP_LXOR, K>(static_cast<A &&>(args)...);
    case OP_BXOR: return call_if<L, OP_BXOR, K>(static_cast<A &&>(args)...);
    case OP_MINLOC: return call_if<L, OP_MINLOC, K>(static_cast<A &&>(args)...);
    case OP_MAXLOC: return call_if<L, OP_MAXLOC, K>(static_cast<A &&>(args)...);
    default: return E_OP;
    }
}

}  // namespace mv2
