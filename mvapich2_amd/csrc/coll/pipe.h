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
// parity p in round k+2 only after waiting (in round k+1) on a flag the
// owner raised after it finished reading round k, and successive calls are
// stream-ordered on every GPU, so two rounds of slots are enough.
#pragma once
#include <type_traits>

#include "kernels_impl.h"

namespace mv2 {

struct NoReduce {};  // instantiation tag: data-movement modes only (AG / BC)

struct Dsts {
    char *p[kMaxRanks + 1];  // nullptr = skip
};

__device__ __forceinline__ char *pslot(char *region, uint64_t par, int src) {
    return region + ((size_t)par * kMaxRanks + (size_t)src) * kPipeSlot;
}

// Block-wide copy of nbytes from src to every non-null destination.
// src and destinations 16-byte aligned; the last partial vector goes bytewise.
template <int U>
__device__ __forceinline__ void blk_copy(const Dsts &d, const char *src, size_t nbytes) {
    const size_t nv = nbytes >> 4;
    const v4u *s = (const v4u *)src;
    size_t i = threadIdx.x;
    for (; i + (size_t)(U - 1) * kThreads < nv; i += (size_t)U * kThreads) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld_nt(s + i + (size_t)u * kThreads);
#pragma unroll
        for (int k = 0; k < kMaxRanks + 1; ++k) {
            if (d.p[k]) {
#pragma unroll
                for (int u = 0; u < U; ++u) st_nt((v4u *)d.p[k] + i + (size_t)u * kThreads, v[u]);
            }
        }
    }
    for (; i < nv; i += kThreads) {
        const v4u v = ld_nt(s + i);
#pragma unroll
        for (int k = 0; k < kMaxRanks + 1; ++k)
            if (d.p[k]) st_nt((v4u *)d.p[k] + i, v);
    }
    const size_t tb = nbytes & 15;
    if (threadIdx.x < tb) {
        const size_t o = (nv << 4) + threadIdx.x;
        const char c = src[o];
#pragma unroll
        for (int k = 0; k < kMaxRanks + 1; ++k)
            if (d.p[k]) d.p[k][o] = c;
    }
}

// Block-wide n-source reduction of nbytes (whole elements) into every
// non-null destination.  src[j] = rank j's operand for this range; `ebase` =
// global element index of the first element (reduction-order owner).
template <class Rd, int U>
__device__ __forceinline__ void blk_reduce(const PipeArgs &a, const char *const (&src)[kMaxRanks], const Dsts &d,
                                           size_t nbytes, size_t ebase) {
    using T = typename Rd::T;
    constexpr int N = 16 / sizeof(T);
    const size_t nv = nbytes >> 4;
    for (size_t i = threadIdx.x; i < nv; i += (size_t)U * kThreads) {
        v4u v[U][kMaxRanks];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t x = i + (size_t)u * kThreads;
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j)
                v[u][j] = (j < a.n && x < nv) ? ld_nt((const v4u *)src[j] + x) : v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t x = i + (size_t)u * kThreads;
            if (x < nv) {
                const v4u r = vreduce_n<Rd>(v[u], a.n, a.tp, ebase + x * N);
#pragma unroll
                for (int k = 0; k < kMaxRanks + 1; ++k)
                    if (d.p[k]) st_nt((v4u *)d.p[k] + x, r);
            }
        }
    }
    const size_t tail = (nbytes & 15) / sizeof(T);
    if (threadIdx.x < tail) {
        const size_t e = nv * N + threadIdx.x;
        T col[kMaxRanks];
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j) col[j] = ((const T *)(j < a.n ? src[j] : src[0]))[e];
        const T r = tree_reduce<Rd>(col, a.n, a.tp.linear, a.tp.pof2, a.tp.rem, elem_owner<Rd>(a.tp, ebase + e));
#pragma unroll
        for (int k = 0; k < kMaxRanks + 1; ++k)
            if (d.p[k]) ((T *)d.p[k])[e] = r;
    }
}

template <class Rd>
__global__ __launch_bounds__(kThreads) void k_pipe(PipeArgs a) {
    const int b = blockIdx.x;
    const int n = a.n, me = a.me;
    const unsigned all = (1u << n) - 1u;
    for (int k = 0; k < a.nrounds; ++k) {
        const uint64_t par = (a.round0 + (uint64_t)k) & 1;
        const uint64_t E = a.epoch0 + 2 * (uint64_t)k;
        const size_t rbase = (size_t)k * a.tseg + (size_t)b * a.tsub;  // segment-relative
        const size_t soff = (size_t)b * a.tsub;                        // slot-relative
        auto rlen = [&](int j) -> size_t {
            return rbase < a.seg_len[j] ? (a.seg_len[j] - rbase < a.tsub ? a.seg_len[j] - rbase : a.tsub) : 0;
        };
        if (a.mode == PIPE_AR || a.mode == PIPE_RS || a.mode == PIPE_RED) {
            if constexpr (!std::is_same<Rd, NoReduce>::value) {
                // P1: scatter my part of every other segment (rotated so blocks spread over links)
                for (int s = 0; s < n - 1; ++s) {
                    const int j = (me + 1 + (b + s) % (n - 1)) % n;
                    const size_t len = rlen(j);
                    if (len) {
                        Dsts d{};
                        d.p[0] = pslot(a.rs_peer.p[j], par, me) + soff;
                        blk_copy<4>(d, a.send + a.seg_off[j] + rbase, len);
                    }
                }
                signal_peers(a.sig_peer, n, me, b, E);
                if (!wait_mask(a.sig_own, all, b, E, a.err, a.timeout)) return;
                // P2: reduce my segment
                const size_t len = rlen(me);
                if (len) {
                    const char *src[kMaxRanks];
#pragma unroll
                    for (int j = 0; j < kMaxRanks; ++j)
                        src[j] = (j == me || j >= n) ? a.send + a.seg_off[me] + rbase
                                                     : pslot(a.rs_peer.p[me], par, j) + soff;
                    Dsts d{};
                    if (a.mode == PIPE_AR) {
                        d.p[kMaxRanks] = a.recv + a.recv_off[me] + rbase;
#pragma unroll
                        for (int j = 0; j < kMaxRanks; ++j)
                            if (j < n && j != me) d.p[j] = pslot(a.ag_peer.p[j], par, me) + soff;
                    } else if (a.mode == PIPE_RS || me == a.root) {
                        d.p[kMaxRanks] = a.recv + a.recv_off[me] + rbase;
                    } else {
                        d.p[0] = pslot(a.ag_peer.p[a.root], par, me) + soff;
                    }
                    blk_reduce<Rd, 1>(a, src, d, len, (a.seg_off[me] + rbase) / (size_t)a.esize);
                }
                if (a.mode == PIPE_RS) continue;
                signal_peers(a.sig_peer, n, me, b, E + 1);
                if (a.mode == PIPE_RED && me != a.root) continue;
                if (!wait_mask(a.sig_own, all, b, E + 1, a.err, a.timeout)) return;
                // P3: gather the other segments' results
                for (int s = 0; s < n - 1; ++s) {
                    const int j = (me + 1 + (b + s) % (n - 1)) % n;
                    const size_t l = rlen(j);
                    if (l) {
                        Dsts d{};
                        d.p[0] = a.recv + a.recv_off[j] + rbase;
                        blk_copy<4>(d, pslot(a.ag_peer.p[me], par, j) + soff, l);
                    }
                }
            }
        } else if (a.mode == PIPE_AG) {
            const size_t len = rlen(me);
            if (len) {
                Dsts d{};
#pragma unroll
                for (int j = 0; j < kMaxRanks; ++j)
                    if (j < n && j != me) d.p[j] = pslot(a.ag_peer.p[j], par, me) + soff;
                if (a.send != a.recv + a.recv_off[me]) d.p[kMaxRanks] = a.recv + a.recv_off[me] + rbase;
                blk_copy<4>(d, a.send + rbase, len);
            }
            signal_peers(a.sig_peer, n, me, b, E);
            if (!wait_mask(a.sig_own, all, b, E, a.err, a.timeout)) return;
            for (int s = 0; s < n - 1; ++s) {
                const int j = (me + 1 + (b + s) % (n - 1)) % n;
                const size_t l = rlen(j);
                if (l) {
                    Dsts d{};
                    d.p[0] = a.recv + a.recv_off[j] + rbase;
                    blk_copy<4>(d, pslot(a.ag_peer.p[me], par, j) + soff, l);
                }
            }
        } else {  // PIPE_BC (send == recv == the buffer, seg_off == recv_off)
            const int root = a.root;
            if (me == root) {
                for (int s = 0; s < n - 1; ++s) {
                    const int j = (me + 1 + (b + s) % (n - 1)) % n;
                    const size_t l = rlen(j);
                    if (l) {
                        Dsts d{};
                        d.p[0] = pslot(a.rs_peer.p[j], par, root) + soff;
                        blk_copy<4>(d, a.send + a.seg_off[j] + rbase, l);
                    }
                }
                const size_t l = rlen(root);
                if (l) {
                    Dsts d{};
#pragma unroll
                    for (int j = 0; j < kMaxRanks; ++j)
                        if (j < n && j != root) d.p[j] = pslot(a.ag_peer.p[j], par, root) + soff;
                    blk_copy<4>(d, a.send + a.seg_off[root] + rbase, l);
                }
                signal_peers(a.sig_peer, n, me, b, E + 1);
                if (!wait_mask(a.sig_own, all, b, E + 1, a.err, a.timeout)) return;
            } else {
                if (!wait_mask(a.sig_own, 1u << root, b, E, a.err, a.timeout)) return;
                const size_t l = rlen(me);
                if (l) {
                    Dsts d{};
                    d.p[kMaxRanks] = a.recv + a.recv_off[me] + rbase;
#pragma unroll
                    for (int j = 0; j < kMaxRanks; ++j)
                        if (j < n && j != me && j != root) d.p[j] = pslot(a.ag_peer.p[j], par, me) + soff;
                    blk_copy<4>(d, pslot(a.rs_peer.p[me], par, root) + soff, l);
                }
                signal_peers(a.sig_peer, n, me, b, E + 1);
                if (!wait_mask(a.sig_own, all, b, E + 1, a.err, a.timeout)) return;
                for (int s = 0; s < n - 1; ++s) {
                    const int j = (me + 1 + (b + s) % (n - 1)) % n;
                    const size_t lj = rlen(j);
                    if (lj) {
                        Dsts d{};
                        d.p[0] = a.recv + a.recv_off[j] + rbase;
                        blk_copy<4>(d, pslot(a.ag_peer.p[me], par, j) + soff, lj);
                    }
                }
            }
        }
    }
}

template <int OP, int K>
struct LPipe {
    static int run(const PipeArgs &a, const LaunchCfg &cfg) {
        hipLaunchKernelGGL((k_pipe<R<OP, K>>), dim3(cfg.grid), dim3(kThreads), 0, cfg.stream, a);
        return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
    }
};

}  // namespace mv2
