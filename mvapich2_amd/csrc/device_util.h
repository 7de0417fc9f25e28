// device_util.h — gfx950 device helpers shared by the op and collective kernels.
//
// Cross-GPU hand-off protocol (one process per GPU, peers' memory mapped with
// hipIpcOpenMemHandle, flags in hipDeviceMallocUncached signal pages):
//   producer: stores -> every wave s_waitcnt vmcnt(0) -> __syncthreads ->
//             lane 0 system-scope release fence (buffer_wbl2) -> asm vmcnt(0)
//             -> relaxed system-scope flag stores (one lane per peer)
//   consumer: one wave polls its own (uncached, local) flag words with
//             never-writing atomics (flag_load: read where the memory is),
//             with s_sleep, bounded by a wall-clock timeout -> lane 0
//             system-scope acquire fence (buffer_inv sc0 sc1: drops stale
//             L1/L2 lines of peer memory) -> __syncthreads -> plain loads.
// Flags carry monotonically increasing 64-bit epochs (never reset), so no
// per-call memset is needed and a stale flag can only read as "not yet".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace mv2 {

constexpr int kMaxRanks = 8;        // device collectives: ranks per node
constexpr int kMaxBlocks = 1024;    // flag slots per (source rank)
constexpr int kThreads = 256;

struct PeerTable {
    const char *p[kMaxRanks];
};
struct PeerTableW {
    char *p[kMaxRanks];
};
struct SigTable {
    uint64_t *p[kMaxRanks];
};

// One reduction program over the n rank operands of an element: registers
// w[j] start as rank j's value; step s computes w[dst[s]] = w[dst[s]] op
// w[src[s]] (dst is the accumulator, the reference's inoutvec); the result is
// w[res].  Any binary reduction tree of an MV2 algorithm compiles to one
// (runtime/orders.cpp).  The fields are uniform over a workgroup range, so
// prog_eval selects registers with uniform compares: no scratch memory.
struct Prog {
    uint8_t nsteps, res;
    uint8_t dst[kMaxRanks - 1];
    uint8_t src[kMaxRanks - 1];
};
// Programs by element block: element e uses p[min(e / blk, nprog - 1)]
// (the pof2 blocks of a recursive-halving reduce-scatter, last block takes
// the remainder, reduce_osu.c:908-910; the n chunks of the ring).
struct ProgSet {
    int32_t nprog;
    int32_t pad;
    uint64_t blk;
    Prog p[kMaxRanks];
};

// Completion word of one blocking call (flag == nullptr: not armed).  The
// last workgroup to finish raises *flag = seq in pinned host memory, so the
// host returns from the MPI call without the kernel-completion signal
// round trip (runtime/coll.cpp finish()).
constexpr int kDoneStride = 1024;  // counter spacing in words (4 KiB: separate memory channels)
constexpr int kDoneSub = 64;       // first-level counters (blockIdx % 64)
constexpr int kDoneCtrs = kDoneSub + 8 + 1;  // + group counters (blockIdx % 8) + groups done; each with an XCD mask
constexpr size_t kDoneBytes = (size_t)kDoneCtrs * kDoneStride * sizeof(uint32_t);
// largest grid whose arrivals block_done's counter fields hold exactly: <= 16384 per sub-counter,
// so the sums stay in their fields for any 4-bit HW_REG_XCC_ID (sum of squares <= 225 x 16384)
constexpr int kDoneMaxGrid = 1 << 20;
// ints in the pinned error word block (wait_mask records a timeout's context there)
constexpr int kErrWords = 64;
struct Done {
    uint32_t *ctr;   // kDoneCtrs 64-bit counters, kDoneStride words apart; all 0 between launches
    uint64_t *flag;  // pinned host words: [0] last completed seq, [1] last seq whose groups were split over XCDs
    uint64_t seq;
};

#ifdef __HIPCC__  // device code below: only in hipcc-compiled translation units
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_nt(v4u *p, v4u v) { __builtin_nontemporal_store(v, p); }
// streamed (read-once) loads: non-temporal.  Measured on MI355X for the 2-read/1-write
// Reduce_local stream (tools/rl_variants.hip): 6.2-6.3 TB/s vs 5.2-5.3 TB/s with plain loads.
__device__ __forceinline__ v4u ld_nt(const v4u *p) { return __builtin_nontemporal_load(p); }
// one element of any kind (complex / pair structs: in the widest aligned words)
template <class T>
__device__ __forceinline__ T ld_nt_elem(const T *p) {
    if constexpr (std::is_arithmetic<T>::value) {
        return __builtin_nontemporal_load(p);
    } else {
        using W = typename std::conditional<sizeof(T) % 8 == 0 && alignof(T) >= 8, uint64_t,
                  typename std::conditional<sizeof(T) % 4 == 0 && alignof(T) >= 4, uint32_t,
                  typename std::conditional<sizeof(T) % 2 == 0 && alignof(T) >= 2, uint16_t, uint8_t>::type>::type>::type;
        W w[sizeof(T) / sizeof(W)];
#pragma unroll
        for (size_t i = 0; i < sizeof(T) / sizeof(W); ++i) w[i] = __builtin_nontemporal_load((const W *)p + i);
        T r;
        __builtin_memcpy(&r, w, sizeof(T));
        return r;
    }
}

__device__ __forceinline__ void flag_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// A flag poll is an atomic that never writes -- a compare-and-swap against a value no epoch reaches
// -- so it is performed where the memory is, and returns the slot as memory holds it.  A plain
// system-scope load was once served a stale copy of the slot for 30 s while memory held the newer
// epoch, and a system-scope invalidate every 200 us did not clear it (profiles/r06/r06al, r06am).
__device__ __forceinline__ uint64_t flag_load(uint64_t *p) {
    uint64_t v = ~0ull;
    __hip_atomic_compare_exchange_strong(p, &v, ~0ull, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return v;
}

// Release this workgroup's prior global stores at system scope and raise
// flag[me][blk] = epoch on every rank in [0, n).  Call from all threads.
// light = true: the data the peers read is in uncached memory, so the
// acknowledged stores (vmcnt(0)) are already visible; skip the L2 writeback.
__device__ __forceinline__ void signal_peers(const SigTable &sig, int n, int me, int blk,
                                             uint64_t epoch, bool light = false) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64) {
        if (threadIdx.x == 0 && !light) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // same wave as the fence: lanes 0..n-1 store after it in program order
        __builtin_amdgcn_wave_barrier();
        if ((int)threadIdx.x < n) flag_store(sig.p[threadIdx.x] + (size_t)me * kMaxBlocks + blk, epoch);
    }
}

// Wait until flag[j][blk] >= epoch for every rank j whose bit is set in
// `mask` (own slot may be included), then acquire at system scope.  Returns
// false (and records *err) on timeout.  Call from all threads; the result is
// block-uniform.
// light = true: every byte handed off lives in this GPU's uncached arena and is
// read with non-temporal loads (L1 bypassed, uncached memory not held in L2),
// so the system-scope acquire (an L1 + L2 invalidate, >= 1.7 us) is skipped;
// the MPI_Init self-test checks the pairing of light release and light acquire.
// On timeout the error word block (pinned host, kErrWords ints) records what was awaited:
// [1] workgroup, [2..3] epoch, [4] mask, [8 + 2j .. 9 + 2j] the last flag value seen from rank j
// (several timed-out workgroups may interleave their records; each field is one of theirs).
__device__ __forceinline__ bool wait_mask(uint64_t *own_sig, unsigned mask, int blk, uint64_t epoch,
                                          int *err, uint64_t timeout_ticks, bool light = false) {
    __shared__ int s_ok;
    if (threadIdx.x < 64) {
        const int j = threadIdx.x;
        bool ok = j >= kMaxRanks || !((mask >> j) & 1u);
        uint64_t seen = 0;
        const uint64_t t0 = wall_clock64();
        bool timed_out = false;
        while (!__all(ok)) {
            if (!ok) {
                seen = flag_load(own_sig + (size_t)j * kMaxBlocks + blk);
                ok = seen >= epoch;
            }
            if (__all(ok)) break;
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > timeout_ticks) { timed_out = true; break; }
        }
        if (timed_out && j < kMaxRanks && ((mask >> j) & 1u)) {
            __hip_atomic_store(err + 8 + 2 * j, (int)(uint32_t)seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(err + 9 + 2 * j, (int)(uint32_t)(seen >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (threadIdx.x == 0) {
            if (timed_out) {
                __hip_atomic_store(err + 1, blk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(err + 2, (int)(uint32_t)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(err + 3, (int)(uint32_t)(epoch >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(err + 4, (int)mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(err, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                s_ok = 0;
            } else {
                if (!light) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                s_ok = 1;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    return s_ok != 0;
}

// wait on every rank in [0, n)
__device__ __forceinline__ bool wait_peers(uint64_t *own_sig, int n, int blk, uint64_t epoch,
                                           int *err, uint64_t timeout_ticks, bool light = false) {
    return wait_mask(own_sig, (1u << n) - 1u, blk, epoch, err, timeout_ticks, light);
}

// Arrive at the call's completion word (all threads of the block).  Each
// block waits for its own stores to be acknowledged and counts itself,
// relaxed, in sub-counter blockIdx % 64 (spreads the arrivals of a large
// grid over 64 addresses); the last arrival of a sub-counter counts it in its
// group blockIdx % 8; the last arrival of a group writes back the L2 of the
// XCD it runs on (one agent-scope release per group, not per block: a release
// per block cost 20-220 us on a 256 MiB Reduce_local) and counts the group;
// the last group resets the counters for the next launch and publishes seq to
// the host at system scope.  Stream-ordered consumers of the result wait for
// the kernel's end anyway; the release makes the data visible to work on other
// streams of this GPU as soon as the host returns.
//
// Blocks b and b + 8 are observed to share an XCD, but HIP promises no
// workgroup -> XCD placement (MI355X_MICROARCH.md "Contract"), and one group's
// release writes back only the XCD it runs on.  So every arrival carries the XCD
// it really ran on (HW_REG_XCC_ID) in the same 64-bit atomic add that counts it:
// the count, the sum of the XCD ids and the sum of their squares.  For m
// arrivals sum^2 <= m * sumsq, with equality exactly when all m ran on one XCD
// (Cauchy-Schwarz), so a counter's last arrival knows whether its blocks shared
// its XCD without one more atomic.  A split sub-counter or group is "split" (it
// adds to the split field of the level above); the last group then also writes
// seq into d.flag[1], and the host completes that call with a stream
// synchronisation (the kernel's end releases every XCD's L2) instead of trusting
// the word (runtime/coll.cpp wait_done).  Fields of a counter word: count bits
// 0-16, sum 17-35, sum of squares 36-57, split subs / groups 58-63 (exact for
// up to 16384 arrivals per sub-counter, i.e. grids up to 1 Mi blocks: the
// launchers' grids stay within kDoneMaxGrid, runtime/world.cpp clamps rl_grid).
constexpr int kDoneSumShift = 17, kDoneSqShift = 36, kDoneSplitShift = 58;
constexpr uint64_t kDoneCntMask = (1ull << kDoneSumShift) - 1;

__device__ __forceinline__ unsigned xcc_id() {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x;
}
// one arrival from XCD x (plus `split` split arrivals of the level below)
__device__ __forceinline__ uint64_t done_arrival(unsigned x, bool split) {
    return 1ull + ((uint64_t)x << kDoneSumShift) + ((uint64_t)(x * x) << kDoneSqShift) +
           (split ? 1ull << kDoneSplitShift : 0ull);
}
// the counter's arrivals did not all run on one XCD, or one of them was split
__device__ __forceinline__ bool done_split(uint64_t v) {
    const uint64_t m = v & kDoneCntMask, sum = (v >> kDoneSumShift) & ((1ull << (kDoneSqShift - kDoneSumShift)) - 1),
                   sq = (v >> kDoneSqShift) & ((1ull << (kDoneSplitShift - kDoneSqShift)) - 1);
    return (v >> kDoneSplitShift) != 0 || sum * sum != m * sq;
}

__device__ __forceinline__ void block_done(const Done &d) {
    if (!d.flag) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (gridDim.x == 1) {
        // one workgroup (small-message one-shot): no counters, no agent fence; the
        // system-scope release of the host word writes back this XCD's L2 itself
        if (threadIdx.x == 0) __hip_atomic_store(d.flag, d.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (threadIdx.x == 0) {
        const unsigned nb = gridDim.x, b = blockIdx.x;
        const unsigned i = b % kDoneSub, x = b & 7u, me = xcc_id();
        const unsigned members = (nb - i + kDoneSub - 1) / kDoneSub;  // blocks with b % 64 == i
        const unsigned nsub = nb < (unsigned)kDoneSub ? nb : (unsigned)kDoneSub;
        const unsigned subs = (nsub - x + 7u) / 8u;                    // sub-counters i < nsub with i % 8 == x
        const unsigned groups = nb < 8u ? nb : 8u;
        uint64_t *sub = (uint64_t *)(d.ctr + i * kDoneStride), *grp = (uint64_t *)(d.ctr + (kDoneSub + x) * kDoneStride),
                 *all = (uint64_t *)(d.ctr + (kDoneSub + 8) * kDoneStride);
        const uint64_t a = done_arrival(me, false);
        const uint64_t vs = __hip_atomic_fetch_add(sub, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + a;
        if ((vs & kDoneCntMask) != members) return;
        const uint64_t ag = done_arrival(me, done_split(vs));
        const uint64_t vg = __hip_atomic_fetch_add(grp, ag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + ag;
        if ((vg & kDoneCntMask) != subs) return;
        // this XCD's L2 written back before its group counts as done.  The wait is explicit: after a
        // returned atomic the compiler drops the s_waitcnt behind buffer_wbl2 (MI355X_MICROARCH.md,
        // compiler hazard), and the next add then overtook the write-back — the host saw the word
        // while another XCD's dirty lines were still in its L2, and a copy engine reading the result
        // (point-to-point copies of a host-driven schedule) read stale bytes (r04x, 12-rank Iallreduce)
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t aa = done_arrival(0, done_split(vg));
        const uint64_t va = __hip_atomic_fetch_add(all, aa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + aa;
        if ((va & kDoneCntMask) != groups) return;
        for (int k = 0; k < kDoneCtrs; ++k)
            __hip_atomic_store((uint64_t *)(d.ctr + k * kDoneStride), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (va >> kDoneSplitShift) __hip_atomic_store(d.flag + 1, d.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(d.flag, d.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// a x b elementwise on one 16-byte vector holding 16/sizeof(T) elements
template <class Rd>
__device__ __forceinline__ v4u vapply(v4u a, v4u b) {
    using T = typename Rd::T;
    constexpr int N = 16 / sizeof(T);
    T ta[N], tb[N];
    __builtin_memcpy(ta, &a, 16);
    __builtin_memcpy(tb, &b, 16);
#pragma unroll
    for (int i = 0; i < N; ++i) ta[i] = Rd::apply(ta[i], tb[i]);
    __builtin_memcpy(&a, ta, 16);
    return a;
}

// ---- n-input reduction tree on one element (n <= 8, all indices constant) ----
// LINEAR   : ((v0 . v1) . v2) ...                (two-level reduce_shmem order; linear == 3 is
//                                                  the flat ring allreduce on rotated sources)
// RING     : v_{n-1} . (... (v2 . (v1 . v0)))    (linear == 2; reduce-scatter ring, rotated sources)
// GROUPED  : (g_0 . g_d) . g_2d ..., g_k = LINEAR over ranks k .. k+d-1 (linear == 5, d in pof2)
// BUTTERFLY: non-pof2 fold w[i] = v[2i+1] . v[2i] for i < rem, then levels
//            m = 1, 2, 4 pairing (j, j+m); the left operand is the subtree
//            containing `owner` (recursive halving / doubling order).
// ORD >= 0 fixes the order at compile time (hot loops: one specialised body per
// order); ORD = -1 reads it from `linear` at run time.
template <class Rd, int ORD = -1>
__device__ __forceinline__ typename Rd::T tree_reduce(const typename Rd::T (&v)[kMaxRanks], int n,
                                                      int linear, int pof2, int rem, int owner) {
    using T = typename Rd::T;
    if constexpr (Rd::kOrderFree) {  // ops/functors.h: every order gives these bits
        T acc = v[0];
#pragma unroll
        for (int i = 1; i < kMaxRanks; ++i)
            if (i < n) acc = Rd::apply(acc, v[i]);
        return acc;
    }
    if (ORD >= 0) linear = ORD;
    if (linear == 2) {
        // RING (MPIR_Reduce_scatter_ring red_scat_osu.c:1121-1141): sources pre-rotated so
        // v[0] = x_{b+1}, v[k] = x_{b+1+k}; each hop's own operand is the accumulator (inout)
        T acc = v[0];
#pragma unroll
        for (int i = 1; i < kMaxRanks; ++i)
            if (i < n) acc = Rd::apply(v[i], acc);
        return acc;
    }
    if (linear == 5) {
        // GROUPED (one-shot only; `pof2` carries the group size d): the two-level degree-d shm
        // tree, mv2_shm_tree_reduce ch3_shmem_coll.c:4302-4340 — the leader of each group of d
        // reduces its members in order, rank 0 then reduces the other leaders in order
        const int d = pof2;
        T acc = v[0], grp = v[0];
        bool first = true;
#pragma unroll
        for (int i = 1; i < kMaxRanks; ++i) {
            if (i < n) {
                if (i % d == 0) {
                    if (!first) acc = Rd::apply(acc, grp);
                    grp = v[i];
                    first = false;
                } else if (first) {
                    acc = Rd::apply(acc, v[i]);
                } else {
                    grp = Rd::apply(grp, v[i]);
                }
            }
        }
        if (!first) acc = Rd::apply(acc, grp);
        return acc;
    }
    if (linear) {
        T acc = v[0];
#pragma unroll
        for (int i = 1; i < kMaxRanks; ++i)
            if (i < n) acc = Rd::apply(acc, v[i]);
        return acc;
    }
    // w[i] = v[i + rem] as a two-stage shifter (selects between constant
    // indices only: a 4-way select chain is turned into a private-memory
    // table lookup by the compiler)
    T w[kMaxRanks];
#pragma unroll
    for (int i = 0; i < kMaxRanks; ++i) w[i] = (rem & 1) ? v[i + 1 < kMaxRanks ? i + 1 : kMaxRanks - 1] : v[i];
#pragma unroll
    for (int i = 0; i < kMaxRanks; ++i) w[i] = (rem & 2) ? w[i + 2 < kMaxRanks ? i + 2 : kMaxRanks - 1] : w[i];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < rem) w[i] = Rd::apply(v[2 * i + 1], v[2 * i]);
#pragma unroll
    for (int m = 1; m < kMaxRanks; m <<= 1) {
        if (m < pof2) {
#pragma unroll
            for (int j = 0; j + m < kMaxRanks; j += 2 * m) {
                if (j + m < pof2) {
                    const bool up = (owner & m) != 0;
                    const T x = up ? w[j + m] : w[j];
                    const T y = up ? w[j] : w[j + m];
                    w[j] = Rd::apply(x, y);
                }
            }
        }
    }
    return w[0];
}

// Evaluate a reduction program on one element's operands.  All register
// indices are compile-time constants; the program's fields only drive
// selects, so w[] stays in VGPRs whatever the program.
template <class Rd>
__device__ __forceinline__ typename Rd::T prog_eval(const typename Rd::T (&v)[kMaxRanks], const Prog &p) {
    using T = typename Rd::T;
    if constexpr (Rd::kOrderFree) {
        // every order gives these bits (ops/functors.h): fold the program's leaves (each register
        // it names is one rank's operand, used once, all in res's tree -- runtime/orders.cpp
        // Sym::compile checks that for every program it builds) in index order
        unsigned leaves = p.nsteps ? 0u : 1u << p.res;
#pragma unroll
        for (int s = 0; s < kMaxRanks - 1; ++s)
            if (s < p.nsteps) leaves |= (1u << p.dst[s]) | (1u << p.src[s]);
        T acc = v[0];
        bool have = false;
#pragma unroll
        for (int j = 0; j < kMaxRanks; ++j)
            if ((leaves >> j) & 1u) {
                acc = have ? Rd::apply(acc, v[j]) : v[j];
                have = true;
            }
        return acc;
    }
    T w[kMaxRanks];
#pragma unroll
    for (int j = 0; j < kMaxRanks; ++j) w[j] = v[j];
    const int ns = p.nsteps;
#pragma unroll
    for (int s = 0; s < kMaxRanks - 1; ++s) {
        if (s < ns) {
            const int d = p.dst[s], q = p.src[s];
            T a = w[0], b = w[0];
#pragma unroll
            for (int j = 1; j < kMaxRanks; ++j) {
                if (d == j) a = w[j];
                if (q == j) b = w[j];
            }
            const T r = Rd::apply(a, b);
#pragma unroll
            for (int j = 0; j < kMaxRanks; ++j)
                if (d == j) w[j] = r;
        }
    }
    T out = w[0];
#pragma unroll
    for (int j = 1; j < kMaxRanks; ++j)
        if (p.res == j) out = w[j];
    return out;
}

__device__ __forceinline__ int prog_block(const ProgSet &ps, size_t e) {
    if (ps.nprog <= 1) return 0;
    const size_t b = e / ps.blk;
    return b >= (size_t)ps.nprog ? ps.nprog - 1 : (int)b;
}

// bit-reverse of b over lg bits (owner newrank of reduce-scatter block b)
__device__ __forceinline__ int brev_bits(int b, int lg) {
    return lg == 0 ? 0 : (int)(__builtin_bitreverse32((uint32_t)b) >> (32 - lg));
}

#endif  // __HIPCC__

}  // namespace mv2
