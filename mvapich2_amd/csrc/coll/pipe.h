// pipe.h — pipelined push collectives over xGMI through IPC-registered arenas.
//
// One kernel moves a whole collective.  The operand is cut into n segments
// (segment j belongs to rank j) and every segment into rounds of `tseg`
// bytes; workgroup b owns the bytes [k*tseg + b*tsub, +tsub) of every segment
// in round k.  All cross-GPU traffic is stores into the destination GPU's
// arena (hipDeviceMallocUncached, exported once at MPI_Init), published with
// the release/flag protocol of device_util.h:
//
//   AR  P1 scatter : my part of segment j  -> rank j's RS slot [par][me]
//       E          : every rank's P1 stores landed
//       P2 reduce  : segment me = op over the n RS slots (own part straight
//                    from sendbuf), in the reference order (tree_reduce);
//                    result -> my recvbuf and rank j's AG slot [par][me]
//       E+1        : every rank's P2 stores landed
//       P3 gather  : AG slot [par][j] -> my recvbuf segment j
//   RS  P1, E, P2 (result -> recvbuf only)
//   RED P1, E, P2 (root keeps its result, others push to the root), E+1,
//       root P3
//   AG  push my contribution to every AG slot [par][me], E, P3
//   BC  root: segment j -> rank j's RS slot, its own segment -> every AG
//       slot; owners forward their segment to every other AG slot (E+1);
//       P3 gather (scatter + allgather broadcast, bcast_osu.c:1905 family)
//
// Slot reuse: round k writes parity (round0+k)&1.  A rank writes a slot of
// parity p in round k+2 only after waiting on a flag the owner raised after
// it finished reading round k (AR/RS/RED: E(k+2) follows the owner's P2(k+1),
// which follows its P3(k) and P2(k)), and successive calls are stream-ordered
// on every GPU, so two rounds of slots are enough.
//
// Release: every byte a peer reads lives in uncached arena memory, so a
// signal only needs the workgroup's stores acknowledged (s_waitcnt vmcnt(0))
// before the flag store; the system-scope release fence (an L2 writeback of
// unrelated dirty lines on every signal) is kept as an option (light = 0).
#pragma once
#include <type_traits>

#include "kernels_impl.h"

namespace mv2 {

struct NoReduce {};  // instantiation tag: data-movement modes only (AG / BC)

struct Dsts {
    char *p[kMaxRanks + 1];  // nullptr = skip
};

// up to kMaxRanks independent copies (len 0 = unused); all pointers 16-byte aligned
struct Jobs {
    const char *src[kMaxRanks];
    char *dst[kMaxRanks];
    size_t len[kMaxRanks];
};

__device__ __forceinline__ char *pslot(char *region, uint64_t par, int src) {
    return region + ((size_t)par * kMaxRanks + (size_t)src) * kPipeSlotStride;
}

// The copy / reduce loops below are software-pipelined: the loads of the next
// 16-byte column are issued before the stores of the current one.  Stores and
// loads share the in-order vmcnt counter on CDNA, so without the prefetch
// every column would wait for the previous column's (remote, xGMI) stores to
// be acknowledged before its own loads could return.

// Block-wide: every job j copies len[j] bytes.  The jobs' 16-byte columns
// form one flat, job-major index space, so each thread keeps U columns (plus
// the next U) in flight whatever the number of jobs (1 peer at n = 2, 7 at 8).
// The job table lives in LDS: a column's job is found by a scan over the
// prefix sums there (dynamically indexed private arrays would go to scratch).
struct JobTable {
    size_t pre[kMaxRanks + 1];
    const char *src[kMaxRanks];
    char *dst[kMaxRanks];
};

__device__ __forceinline__ void job_addr(const JobTable &t, size_t f, const v4u *&s, v4u *&d) {
    int j = 0;
    for (int k = 1; k < kMaxRanks; ++k) j = f >= t.pre[k] ? k : j;
    s = (const v4u *)t.src[j] + (f - t.pre[j]);
    d = (v4u *)t.dst[j] + (f - t.pre[j]);
}

// LocalDst: destinations are this GPU's own buffers -> plain stores (the HBM
// write path the Reduce_local sweep measured fastest); arena destinations on
// peers keep non-temporal stores.
// head bytes of a range before its first 16-byte boundary (src and dst share the alignment)
__device__ __forceinline__ size_t head_bytes(const char *p, size_t len) {
    const size_t h = (16 - ((uintptr_t)p & 15)) & 15;
    return h < len ? h : len;
}

template <bool LocalDst>
__device__ __forceinline__ void blk_copy_jobs(const Jobs &jb, bool rnt = true) {
    constexpr int U = 4;
    __shared__ JobTable t;
    __syncthreads();  // previous users of the table are done
    if (threadIdx.x == 0) {
        size_t acc = 0;
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j) {
            const size_t h = jb.len[j] ? head_bytes(jb.src[j], jb.len[j]) : 0;
            t.pre[j] = acc;
            t.src[j] = jb.src[j] + h;
            t.dst[j] = jb.dst[j] + h;
            acc += (jb.len[j] - h) >> 4;
        }
        t.pre[kMaxRanks] = acc;
    }
    __syncthreads();
    const size_t NV = t.pre[kMaxRanks];
    size_t f = threadIdx.x;
    if (f < NV) {
        v4u cur[U], nxt[U];
        const v4u *s;
        v4u *d;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t fu = f + (size_t)u * kPipeThreads;
            if (fu < NV) {
                job_addr(t, fu, s, d);
                cur[u] = ld_nt(s);
            }
        }
        for (;;) {
            const size_t fn = f + (size_t)U * kPipeThreads;
            const bool more = fn < NV;
            if (more) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const size_t fu = fn + (size_t)u * kPipeThreads;
                    if (fu < NV) {
                        job_addr(t, fu, s, d);
                        nxt[u] = ld_nt(s);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t fu = f + (size_t)u * kPipeThreads;
                if (fu < NV) {
                    job_addr(t, fu, s, d);
                    if (LocalDst || !rnt) *d = cur[u];
                    else st_nt(d, cur[u]);
                }
            }
            if (!more) break;
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
            f = fn;
        }
    }
    if (threadIdx.x < 32) {  // lanes 0-15: the head, 16-31: the tail of every job
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j) {
            if (!jb.len[j]) continue;
            const size_t h = head_bytes(jb.src[j], jb.len[j]);
            const size_t body = (jb.len[j] - h) & ~(size_t)15;
            const size_t o = threadIdx.x < 16 ? threadIdx.x : h + body + (threadIdx.x - 16);
            if (threadIdx.x < 16 ? o < h : o < jb.len[j])
                jb.dst[j][o] = __builtin_nontemporal_load(jb.src[j] + o);
        }
    }
}

// Block-wide copy of nbytes from one source to every non-null destination.
// src and every destination share the same alignment mod 16: a scalar head up to the
// first 16-byte boundary, then the 16-byte body, then the tail.
__device__ __forceinline__ void blk_copy_multi(const Dsts &dd, const char *src0, size_t nbytes0, bool rnt = true) {
    constexpr int U = 4;
    const size_t h = head_bytes(src0, nbytes0);
    if (threadIdx.x < h) {
        const char c = __builtin_nontemporal_load(src0 + threadIdx.x);
#pragma unroll
        for (int k = 0; k < kMaxRanks + 1; ++k)
            if (dd.p[k]) dd.p[k][threadIdx.x] = c;
    }
    Dsts d = dd;
#pragma unroll
    for (int k = 0; k < kMaxRanks + 1; ++k)
        if (d.p[k]) d.p[k] += h;
    const char *src = src0 + h;
    const size_t nbytes = nbytes0 - h;
    const size_t nv = nbytes >> 4;
    const v4u *s = (const v4u *)src;
    size_t x = threadIdx.x;
    if (x < nv) {
        v4u cur[U], nxt[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (x + (size_t)u * kPipeThreads < nv) cur[u] = ld_nt(s + x + (size_t)u * kPipeThreads);
        for (;;) {
            const size_t xn = x + (size_t)U * kPipeThreads;
            const bool more = xn < nv;
            if (more) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (xn + (size_t)u * kPipeThreads < nv) nxt[u] = ld_nt(s + xn + (size_t)u * kPipeThreads);
            }
#pragma unroll
            for (int k = 0; k < kMaxRanks + 1; ++k) {
                if (d.p[k]) {
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (x + (size_t)u * kPipeThreads < nv) {
                            v4u *q = (v4u *)d.p[k] + x + (size_t)u * kPipeThreads;
                            if (k == kMaxRanks || !rnt) *q = cur[u];  // own recv buffer / plain remote stores
                            else st_nt(q, cur[u]);
                        }
                }
            }
            if (!more) break;
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
            x = xn;
        }
    }
    const size_t tb = nbytes & 15;
    if (threadIdx.x < tb) {
        const size_t o = (nv << 4) + threadIdx.x;
        const char c = __builtin_nontemporal_load(src + o);
#pragma unroll
        for (int k = 0; k < kMaxRanks + 1; ++k)
            if (d.p[k]) d.p[k][o] = c;
    }
}

// Block-wide n-source reduction of nbytes (whole elements) into every
// non-null destination.  src[j] = rank j's operand for this range; `ebase` =
// global element index of the first element (reduction-order owner).
// NM: operand columns held in registers (4 when n <= 4: half the load buffers, so
// the two-column unroll fits without scratch).
template <class Rd, int U, int ORD, int NM = kMaxRanks>
__device__ __forceinline__ void blk_reduce(const PipeArgs &a, const char *const (&src)[kMaxRanks], const Dsts &d,
                                           size_t nbytes, size_t ebase) {
    using T = typename Rd::T;
    constexpr int N = 16 / sizeof(T);
    const size_t nv = nbytes >> 4;
    // butterfly owner / program block: constant over a range inside one block (all but at
    // most nblocks-1 ranges of a call), so the per-vector 64-bit division is hoisted out
    // of the loop.  Program order reads the programs in place (a.tp), never a copy.
    const TreeParams &tpa = a.tp;
    TreeParams tp;
    int fb = -1;
    if constexpr (ORD == 4) {
        if (nbytes >= sizeof(T)) {
            const int b0 = prog_block(tpa.ps, ebase), b1 = prog_block(tpa.ps, ebase + nbytes / sizeof(T) - 1);
            if (b0 == b1) fb = b0;
        }
    } else {
        tp = a.tp;
        if (ORD == 0 && tp.owner_fixed < 0 && nbytes >= sizeof(T)) {
            const int o0 = elem_owner<Rd>(tp, ebase), o1 = elem_owner<Rd>(tp, ebase + nbytes / sizeof(T) - 1);
            if (o0 == o1) tp.owner_fixed = o0;
        }
    }
    size_t x = threadIdx.x;
    if (x < nv) {
        v4u cur[U][NM], nxt[U][NM];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t xu = x + (size_t)u * kPipeThreads;
#pragma unroll
            for (int j = 0; j < NM; ++j)
                cur[u][j] = (j < a.n && xu < nv) ? ld_nt((const v4u *)src[j] + xu) : v4u{0, 0, 0, 0};
        }
        for (;;) {
            const size_t xn = x + (size_t)U * kPipeThreads;
            const bool more = xn < nv;
            if (more) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const size_t xu = xn + (size_t)u * kPipeThreads;
#pragma unroll
                    for (int j = 0; j < NM; ++j)
                        nxt[u][j] = (j < a.n && xu < nv) ? ld_nt((const v4u *)src[j] + xu) : v4u{0, 0, 0, 0};
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t xu = x + (size_t)u * kPipeThreads;
                if (xu < nv) {
                    v4u col[kMaxRanks];
#pragma unroll
                    for (int j = 0; j < kMaxRanks; ++j) col[j] = j < NM ? cur[u][j < NM ? j : 0] : v4u{0, 0, 0, 0};
                    v4u r;
                    if constexpr (ORD == 4) r = vreduce_n<Rd, 4>(col, a.n, tpa, ebase + xu * N, fb);
                    else r = vreduce_n<Rd, ORD>(col, a.n, tp, ebase + xu * N);
#pragma unroll
                    for (int k = 0; k < kMaxRanks + 1; ++k)
                        if (d.p[k]) {
                            if (k == kMaxRanks || !a.rnt) ((v4u *)d.p[k])[xu] = r;  // own recv / plain remote
                            else st_nt((v4u *)d.p[k] + xu, r);
                        }
                }
            }
            if (!more) break;
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < NM; ++j) cur[u][j] = nxt[u][j];
            x = xn;
        }
    }
    const size_t tail = (nbytes & 15) / sizeof(T);
    if (threadIdx.x < tail) {
        const size_t e = nv * N + threadIdx.x;
        T col[kMaxRanks];
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j) col[j] = ld_nt_elem((const T *)(j < a.n ? src[j] : src[0]) + e);
        T r;
        if constexpr (ORD == 4) r = prog_eval<Rd>(col, tpa.ps.p[prog_block(tpa.ps, ebase + e)]);
        else r = tree_reduce<Rd, ORD>(col, a.n, tp.linear, tp.pof2, tp.rem, elem_owner<Rd>(tp, ebase + e));
#pragma unroll
        for (int k = 0; k < kMaxRanks + 1; ++k)
            if (d.p[k]) ((T *)d.p[k])[e] = r;
    }
}

// Scalar reduction of the first nbytes (< 16, whole elements) of a range whose start is not
// 16-byte aligned, in the call's order; ebase = global index of the first element.
template <class Rd, bool PROG>
__device__ __forceinline__ void blk_reduce_head(const PipeArgs &a, const char *const (&src)[kMaxRanks], const Dsts &d,
                                                size_t nbytes, size_t ebase) {
    using T = typename Rd::T;
    const size_t cnt = nbytes / sizeof(T);
    if (threadIdx.x >= cnt) return;
    const size_t e = threadIdx.x;
    T col[kMaxRanks];
#pragma unroll
    for (int j = 0; j < kMaxRanks; ++j) col[j] = ld_nt_elem((const T *)(j < a.n ? src[j] : src[0]) + e);
    T r;
    if constexpr (PROG) {
        r = prog_eval<Rd>(col, a.tp.ps.p[prog_block(a.tp.ps, ebase + e)]);
    } else {
        const TreeParams &tp = a.tp;
        r = tree_reduce<Rd>(col, a.n, tp.linear, tp.pof2, tp.rem, elem_owner<Rd>(tp, ebase + e));
    }
#pragma unroll
    for (int k = 0; k < kMaxRanks + 1; ++k)
        if (d.p[k]) ((T *)d.p[k])[e] = r;
}

__device__ __forceinline__ size_t range_len(const PipeArgs &a, int j, size_t rbase) {
    return rbase < a.seg_len[j] ? (a.seg_len[j] - rbase < a.tsub ? a.seg_len[j] - rbase : a.tsub) : 0;
}

// P3: my AG slots [par][j] -> recv segment j, for every j != me (and != skip)
__device__ __forceinline__ void gather_slots(const PipeArgs &a, uint64_t par, size_t rbase, size_t soff, int skip) {
    Jobs jb{};
#pragma unroll
    for (int j = 0; j < kMaxRanks; ++j) {
        if (j < a.n && j != a.me && j != skip) {
            jb.src[j] = pslot(a.ag_peer.p[a.me], par, j) + soff + (a.seg_off[j] & 15);
            jb.dst[j] = a.recv + a.recv_off[j] + rbase;
            jb.len[j] = range_len(a, j, rbase);
        }
    }
    blk_copy_jobs<true>(jb);
}

// P1 of round k: my part of every other segment -> its owner's RS slot [par][me]
// (all n-1 links at once)
__device__ __forceinline__ void scatter_round(const PipeArgs &a, uint64_t round0, int k) {
    const uint64_t par = (round0 + (uint64_t)k) & 1;
    const size_t rbase = (size_t)k * a.tseg + (size_t)blockIdx.x * a.tsub;
    const size_t soff = (size_t)blockIdx.x * a.tsub;
    Jobs jb{};
#pragma unroll
    for (int j = 0; j < kMaxRanks; ++j) {
        if (j < a.n && j != a.me) {
            jb.src[j] = a.send + a.seg_off[j] + rbase;
            jb.dst[j] = pslot(a.rs_peer.p[j], par, a.me) + soff + (a.seg_off[j] & 15);
            jb.len[j] = range_len(a, j, rbase);
        }
    }
    blk_copy_jobs<false>(jb, a.rnt != 0);
}

// P2 of round k: reduce my segment's range from the n RS slots (own operand
// straight from sendbuf); AR: result -> recv + every peer's AG slot [par][me];
// RS: -> recv; RED: root -> recv, others -> the root's AG slot [par][me]
// PROG: the program-order variant (tp.linear == 4) is a kernel of its own so
// that its register demand never lowers the occupancy of the hot ring /
// butterfly kernel.
// (op, kind) pairs whose pipelined reduction keeps the n <= 4 body with four operand columns and
// two vectors in flight per thread (more loads outstanding per wave; the 2-rank 256 MiB allreduce
// busbw rose with it, r02): the fp SUM / MAX / MIN and the DOUBLE_INT MAXLOC / MINLOC of the
// benchmarks (configs[1]-[4]; DOUBLE_INT MAXLOC at 2 shared ranks: 445 GB/s wide, 401 GB/s eight
// columns, r05a).  Every other pair runs the eight-column body at every n, which halves its share of
// libmpi.so's code objects.
template <class Rd> struct WidePipe : std::false_type {};
template <int OP, int K>
struct WidePipe<R<OP, K, void>>
    : std::integral_constant<bool, ((K == K_F32 || K == K_F64) && (OP == OP_SUM || OP == OP_MAX || OP == OP_MIN)) ||
                                       (K == K_P_DOUBLEINT && (OP == OP_MAXLOC || OP == OP_MINLOC))> {};

template <class Rd, bool PROG>
__device__ __forceinline__ void reduce_round(const PipeArgs &a, uint64_t round0, int k) {
    const uint64_t par = (round0 + (uint64_t)k) & 1;
    const size_t rbase = (size_t)k * a.tseg + (size_t)blockIdx.x * a.tsub;
    const size_t soff = (size_t)blockIdx.x * a.tsub;
    const int me = a.me;
    const size_t len = range_len(a, me, rbase);
    if (!len) return;
    const size_t mis = a.seg_off[me] & 15;  // segment misalignment, kept in the slots
    const char *src[kMaxRanks];
    if (a.tp.linear == 2) {
        // ring order: source k is rank me+1+k (mod n), so the chain ends with my own operand
#pragma unroll
        for (int k = 0; k < kMaxRanks; ++k) {
            int j = me + 1 + k;
            while (j >= a.n) j -= a.n;
            src[k] = (k >= a.n || j == me) ? a.send + a.seg_off[me] + rbase : pslot(a.rs_peer.p[me], par, j) + soff + mis;
        }
    } else if (a.tp.linear == 3) {
        // flat ring allreduce (MPIR_Allreduce_pt2pt_ring_MV2 allreduce_osu.c:3925-3958): segment
        // me is ring chunk me, which starts at rank me and gathers rank me+k at hop k with the
        // received partial as the accumulator -> linear order over sources rotated by me
#pragma unroll
        for (int k = 0; k < kMaxRanks; ++k) {
            int j = me + k;
            while (j >= a.n) j -= a.n;
            src[k] = (k >= a.n || j == me) ? a.send + a.seg_off[me] + rbase : pslot(a.rs_peer.p[me], par, j) + soff + mis;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j)
            src[j] = (j == me || j >= a.n) ? a.send + a.seg_off[me] + rbase : pslot(a.rs_peer.p[me], par, j) + soff + mis;
    }
    Dsts d{};
    if (a.mode == PIPE_AR) {
        d.p[kMaxRanks] = a.recv + a.recv_off[me] + rbase;
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j)
            if (j < a.n && j != me) d.p[j] = pslot(a.ag_peer.p[j], par, me) + soff + mis;
    } else if (a.mode == PIPE_RS || me == a.root) {
        d.p[kMaxRanks] = a.recv + a.recv_off[me] + rbase;
    } else {
        d.p[0] = pslot(a.ag_peer.p[a.root], par, me) + soff + mis;
    }
    size_t e0 = (a.seg_off[me] + rbase) / (size_t)a.esize;
    size_t body = len;
    if (mis) {
        // scalar head up to the first 16-byte boundary (whole elements: extents are powers of two
        // <= 16, so the misalignment is a multiple of the extent), then the aligned body
        const size_t h = (16 - mis) < len ? (16 - mis) : len;
        blk_reduce_head<Rd, PROG>(a, src, d, h, (size_t)((int64_t)e0 + (PROG ? a.eshift : 0)));
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j) src[j] += h;
#pragma unroll
        for (int k = 0; k < kMaxRanks + 1; ++k)
            if (d.p[k]) d.p[k] += h;
        e0 += h / (size_t)a.esize;
        body = len - h;
        if (!body) return;
    }
    const size_t len_body = body;
    // fewer sources -> more columns per thread, so >= 4 loads stay in flight
    // one specialised loop per (unroll, order); the order is uniform over the call
    if constexpr (Rd::kOrderFree) {  // any order gives the same bits: the LINEAR body only
        if (a.n <= 4) blk_reduce<Rd, 2, 1, 4>(a, src, d, len_body, e0);
        else blk_reduce<Rd, 1, 1>(a, src, d, len_body, e0);
    } else if constexpr (PROG) {
        blk_reduce<Rd, 1, 4>(a, src, d, len_body, (size_t)((int64_t)e0 + a.eshift));
    } else if constexpr (!WidePipe<Rd>::value) {
        if (a.tp.linear == 2) blk_reduce<Rd, 1, 2>(a, src, d, len_body, e0);
        else if (a.tp.linear) blk_reduce<Rd, 1, 1>(a, src, d, len_body, e0);
        else blk_reduce<Rd, 1, 0>(a, src, d, len_body, e0);
    } else if (a.n <= 4) {
        if (a.tp.linear == 2) blk_reduce<Rd, 2, 2, 4>(a, src, d, len_body, e0);
        else if (a.tp.linear) blk_reduce<Rd, 2, 1, 4>(a, src, d, len_body, e0);
        else blk_reduce<Rd, 2, 0, 4>(a, src, d, len_body, e0);
    } else {
        if (a.tp.linear == 2) blk_reduce<Rd, 1, 2>(a, src, d, len_body, e0);
        else if (a.tp.linear) blk_reduce<Rd, 1, 1>(a, src, d, len_body, e0);
        else blk_reduce<Rd, 1, 0>(a, src, d, len_body, e0);
    }
}

template <class Rd, bool PROG = false>
__device__ __forceinline__ void pipe_body(const PipeArgs &a, uint64_t epoch0, uint64_t round0) {
    const int b = blockIdx.x;
    const int n = a.n, me = a.me;
    const unsigned all = (1u << n) - 1u;
    if (a.mode == PIPE_AR || a.mode == PIPE_RS || a.mode == PIPE_RED) {
        if constexpr (!std::is_same<Rd, NoReduce>::value) {
            // Rounds overlap: the scatter of round k+1 runs while the peers finish
            // round k's reduction, and round k's gather follows it, so neither flag
            // wait sits on an idle workgroup.
            //   P1(0) E(0) | wait E(k); P2(k); E(k)+1; P1(k+1); E(k+1); wait E(k)+1; P3(k) |
            const bool gathers = a.mode == PIPE_AR || (a.mode == PIPE_RED && me == a.root);
            if (a.nrounds > 0) {
                scatter_round(a, round0, 0);
                signal_peers(a.sig_peer, n, me, b, epoch0, a.light);
            }
            for (int k = 0; k < a.nrounds; ++k) {
                const uint64_t E = epoch0 + 2 * (uint64_t)k;
                if (!wait_mask(a.sig_own, all, b, E, a.err, a.timeout, a.light != 0)) return;
                reduce_round<Rd, PROG>(a, round0, k);
                if (a.mode != PIPE_RS) signal_peers(a.sig_peer, n, me, b, E + 1, a.light);
                if (k + 1 < a.nrounds) {
                    scatter_round(a, round0, k + 1);
                    signal_peers(a.sig_peer, n, me, b, E + 2, a.light);
                }
                if (!gathers) continue;
                if (!wait_mask(a.sig_own, all, b, E + 1, a.err, a.timeout, a.light != 0)) return;
                const size_t rbase = (size_t)k * a.tseg + (size_t)b * a.tsub;
                gather_slots(a, (round0 + (uint64_t)k) & 1, rbase, (size_t)b * a.tsub, -1);
            }
        }
        return;
    }
    for (int k = 0; k < a.nrounds; ++k) {
        const uint64_t par = (round0 + (uint64_t)k) & 1;
        const uint64_t E = epoch0 + 2 * (uint64_t)k;
        const size_t rbase = (size_t)k * a.tseg + (size_t)b * a.tsub;  // segment-relative
        const size_t soff = (size_t)b * a.tsub;                        // slot-relative
        auto rlen = [&](int j) -> size_t { return range_len(a, j, rbase); };
        if (a.mode == PIPE_AG) {
            const size_t len = rlen(me);
            if (len) {
                Dsts d{};
#pragma unroll
                for (int j = 0; j < kMaxRanks; ++j)
                    if (j < n && j != me) d.p[j] = pslot(a.ag_peer.p[j], par, me) + soff + (a.seg_off[me] & 15);
                if (a.send != a.recv + a.recv_off[me]) d.p[kMaxRanks] = a.recv + a.recv_off[me] + rbase;
                blk_copy_multi(d, a.send + rbase, len, a.rnt != 0);
            }
            signal_peers(a.sig_peer, n, me, b, E, a.light);
            if (!wait_mask(a.sig_own, all, b, E, a.err, a.timeout, a.light != 0)) return;
            gather_slots(a, par, rbase, soff, -1);
        } else {  // PIPE_BC (send == recv == the buffer, seg_off == recv_off)
            const int root = a.root;
            if (me == root) {
                {
                    Jobs jb{};
#pragma unroll
                    for (int j = 0; j < kMaxRanks; ++j) {
                        if (j < n && j != root) {
                            jb.src[j] = a.send + a.seg_off[j] + rbase;
                            jb.dst[j] = pslot(a.rs_peer.p[j], par, root) + soff;
                            jb.len[j] = rlen(j);
                        }
                    }
                    blk_copy_jobs<false>(jb, a.rnt != 0);
                }
                const size_t l = rlen(root);
                if (l) {
                    Dsts d{};
#pragma unroll
                    for (int j = 0; j < kMaxRanks; ++j)
                        if (j < n && j != root) d.p[j] = pslot(a.ag_peer.p[j], par, root) + soff;
                    blk_copy_multi(d, a.send + a.seg_off[root] + rbase, l, a.rnt != 0);
                }
                signal_peers(a.sig_peer, n, me, b, E + 1, a.light);
                if (!wait_mask(a.sig_own, all, b, E + 1, a.err, a.timeout, a.light != 0)) return;
            } else {
                if (!wait_mask(a.sig_own, 1u << root, b, E, a.err, a.timeout, a.light != 0)) return;
                const size_t l = rlen(me);
                if (l) {
                    Dsts d{};
                    d.p[kMaxRanks] = a.recv + a.recv_off[me] + rbase;
#pragma unroll
                    for (int j = 0; j < kMaxRanks; ++j)
                        if (j < n && j != me && j != root) d.p[j] = pslot(a.ag_peer.p[j], par, me) + soff;
                    blk_copy_multi(d, pslot(a.rs_peer.p[me], par, root) + soff, l, a.rnt != 0);
                }
                signal_peers(a.sig_peer, n, me, b, E + 1, a.light);
                if (!wait_mask(a.sig_own, all, b, E + 1, a.err, a.timeout, a.light != 0)) return;
                gather_slots(a, par, rbase, soff, -1);
            }
        }
    }
}

template <class Rd, bool PROG = false>
__global__ __launch_bounds__(kPipeThreads) void k_pipe(PipeArgs a) {
    uint64_t epoch0 = a.epoch0, round0 = a.round0;
    if (a.dseq) {  // graph lane: this replay's base, read before any workgroup can advance it
        const SeqBase q = dseq_read(a.dseq);
        epoch0 = q.epoch + 1;
        round0 = q.round;
    }
    pipe_body<Rd, PROG>(a, epoch0, round0);
    if (a.dseq) dseq_advance(a.dseq, 2 * (uint64_t)a.nrounds, (uint64_t)a.nrounds, 0);
    block_done(a.done);
}

template <int OP, int K>
struct LPipe {
    static int run(const PipeArgs &a, const LaunchCfg &cfg) {
        if constexpr (R<OP, K>::kOrderFree)
            hipLaunchKernelGGL((k_pipe<R<OP, K>, false>), dim3(cfg.grid), dim3(kPipeThreads), 0, cfg.stream, a);
        else if (a.tp.linear == 4)
            hipLaunchKernelGGL((k_pipe<R<OP, K>, true>), dim3(cfg.grid), dim3(kPipeThreads), 0, cfg.stream, a);
        else
            hipLaunchKernelGGL((k_pipe<R<OP, K>, false>), dim3(cfg.grid), dim3(kPipeThreads), 0, cfg.stream, a);
        return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
    }
};

}  // namespace mv2
