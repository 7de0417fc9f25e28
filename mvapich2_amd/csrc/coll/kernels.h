// kernels.h — host-side launch interface of the HIP kernels (C++ only, internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../device_util.h"

namespace mv2 {

struct TreeParams {
    int linear;      // 1: LINEAR, 0: BUTTERFLY, 2: RS ring, 3: AR ring (rotated), 4: PROGRAM (ps),
                     // 5: GROUPED (one-shot kernel only; group size in pof2)
    int pof2, rem, lg;
    int owner_fixed; // >= 0: fixed owner newrank; -1: reduce-scatter block owner
    size_t rs_blk;   // elements per reduce-scatter block (count / pof2)
    ProgSet ps;      // linear == 4
};

// Sequence numbers of the graph lane (coll.cpp, HIP graph capture): a captured kernel cannot
// carry host-assigned flag epochs and slot parities, because every replay would reuse them, so
// graph-lane kernels read their base here when they start and the last workgroup to finish
// advances it for the next call (uncached device memory; one block per process).
struct DevSeq {
    uint64_t epoch;   // last flag epoch used
    uint64_t round;   // pipeline rounds issued (slot parity)
    uint64_t os;      // one-shot calls issued (arena half)
    uint32_t arrive;  // workgroups of the running kernel that have finished
    uint32_t pad[9];
};

struct OneShotArgs {
    const char *send;
    char *recv;
    PeerTableW arena_peer;   // peers' arena (this call's parity half); my slot at + me*slot_bytes
    const char *arena_own;   // my arena (same parity); rank j's slot at + j*slot_bytes
    SigTable sig_peer;
    uint64_t *sig_own;
    size_t count, nvec, slot_bytes;
    int n, me;
    TreeParams tp;
    uint64_t epoch;
    int *err;
    uint64_t timeout;
    int light;    // 1: signal without the L2 writeback (peers read only uncached arena data)
    Done done;
    // graph lane (HIP graph capture): epoch and arena half come from the device sequence
    // block at run time (arena_peer / arena_own then point at half 0; `half` = bytes per half)
    DevSeq *dseq;
    size_t half;
    // reduce-scatter (rs = 1): rank j reduces only elements [wlo[j], wlo[j] + wcnt[j]) of the
    // operand (wlo[j] a multiple of 16 / sizeof(T)) into its recv from the start; each rank
    // pushes every peer only that peer's block (coll/kernels_impl.h k_oneshot_rs)
    int rs;
    size_t wlo[kMaxRanks], wcnt[kMaxRanks];
    // data movement (k_oneshot_mv, coll/dispatch.hip): 0 = reducing; 1 = allgather (count bytes per
    // rank from send, rank j's block to recv + j * pitch); 2 = broadcast (count bytes of recv from root)
    int mv, root;
    size_t pitch;
};

// ---------------------------------------------------------------------------
// Pipelined push collectives through IPC-registered arenas (coll/pipe.h).
// User buffers are never mapped by peers: every cross-GPU byte is a store
// into a library-owned, uncached arena slot of the destination GPU, so
// applications may free or reuse their buffers as soon as a call returns.
// ---------------------------------------------------------------------------
enum PipeMode : int {
    PIPE_AR = 0,   // allreduce: scatter -> reduce own segment + push -> gather
    PIPE_RS = 1,   // reduce-scatter: scatter -> reduce own segment into recv
    PIPE_RED = 2,  // reduce to root: scatter -> reduce -> push to root -> root gathers
    PIPE_AG = 3,   // allgather: push own contribution -> gather
    PIPE_BC = 4,   // broadcast: root scatters segments -> owners push -> gather
};

// Arena layout per rank and region (RS region, AG region):
//   [parity 0..1][source rank 0..kMaxRanks-1][kPipeSlotStride bytes]
// Round k of a call uses parity (round0 + k) & 1; block b moves the bytes
// [k*tseg + b*tsub, +tsub) of every segment, stored at slot offset
// b*tsub + (segment offset mod 16): a segment that starts off a 16-byte
// boundary (ring chunks of n = 3, 5, 6 ...) keeps its misalignment in the
// slot, so every copy and reduction pairs addresses of equal alignment
// (scalar head, 16-byte body, scalar tail).  The stride leaves room for it.
constexpr int kPipeThreads = 512;                // 8 waves per workgroup
constexpr int kPipeMaxGrid = 256;                // one workgroup per CU
constexpr size_t kPipeMaxSub = (size_t)128 << 10;
constexpr size_t kPipeSlot = (size_t)kPipeMaxGrid * kPipeMaxSub;  // 32 MiB of data
constexpr size_t kPipeSlotStride = kPipeSlot + 256;
constexpr size_t kPipeRegion = 2 * (size_t)kMaxRanks * kPipeSlotStride;

struct PipeArgs {
    int mode, n, me, root;
    const char *send;               // AR/RS/RED: full operand; AG: my contribution; BC: the buffer
    char *recv;                     // destination base
    size_t seg_off[kMaxRanks];      // byte offset of segment j in `send` (16-byte aligned)
    size_t seg_len[kMaxRanks];      // bytes of segment j
    size_t recv_off[kMaxRanks];     // byte offset in `recv` where segment j lands (16-byte aligned)
    PeerTableW rs_peer;             // rank j's RS region (mapped); entry me = my own
    PeerTableW ag_peer;             // rank j's AG region (mapped); entry me = my own
    size_t tseg, tsub;              // bytes per segment per round / per block per segment per round
    uint64_t round0;                // global round counter at launch (slot parity)
    int nrounds;
    int esize;                      // element extent (reducing modes)
    int64_t eshift;                 // program order: global element index = (seg_off[me] + r) / esize + eshift
    SigTable sig_peer;
    uint64_t *sig_own;
    uint64_t epoch0;                // round k uses epochs epoch0 + 2k and epoch0 + 2k + 1
    int light;                      // 1: signal without the system-scope L2 writeback (uncached data)
    int rnt;                        // 1: non-temporal stores into peers' arenas, 0: plain (MPI_Init autotune)
    TreeParams tp;
    int *err;
    uint64_t timeout;
    Done done;
    DevSeq *dseq;                   // graph lane: epoch0 / round0 read from here at run time
};

struct LaunchCfg {
    int grid;
    int unroll;
    hipStream_t stream;
    int cus = 256;    // compute units of the device
    int nshare = 1;   // max ranks sharing one GPU (same on every rank)
    Done done{};      // completion word (reduce_local)
    size_t tiny_max = 0;  // reduce_local: operands up to this many bytes take the one-wave kernel
};

// Grid cap for `per_cu` blocks per CU when `nshare` ranks share the GPU.
// Blocks are dealt round-robin over the 8 XCDs from an XCD that is not fixed
// (MI355X_MICROARCH.md, Workgroup dispatch), so a grid g puts up to ceil(g/8)
// blocks on one XCD; with nshare spinning kernels every XCD must hold nshare of
// those.  The cap is therefore 8 * floor(per_cu * cus_per_xcd / nshare): 256
// at nshare 1, 48 (not 51) at 5 ranks, where 51-block grids could deadlock.
inline int xcd_fair_cap(int per_cu, int cus, int nshare) {
    const int xcds = (cus >= 64 && cus % 8 == 0) ? 8 : 1;
    const int per_xcd = per_cu * (cus / xcds) / (nshare > 0 ? nshare : 1);
    return (per_xcd < 1 ? 1 : per_xcd) * xcds;
}

// Workgroups that are guaranteed co-resident for a kernel (the per-workgroup
// cross-GPU flags need block b of every rank running together).  The
// occupancy API can over-report by one block per CU (MI355X_MICROARCH.md,
// Residency), so one block per CU is held back.
inline int resident_grid(const void *kernel, const LaunchCfg &cfg) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, kThreads, 0) != hipSuccess || nb < 1) nb = 1;
    nb = nb > 1 ? nb - 1 : 1;
    return xcd_fair_cap(nb, cfg.cus, cfg.nshare);
}

// all return an MPI error class (0 = launched)
int launch_reduce_local(int op, int kind, const void *in, void *inout, size_t count, size_t esize,
                        const LaunchCfg &cfg);
int launch_reduce_n(int op, int kind, const void *const *srcs, int n, void *dst, size_t count,
                    size_t esize, const TreeParams &tp, const LaunchCfg &cfg);
int launch_oneshot(int op, int kind, const OneShotArgs &a, size_t esize, const LaunchCfg &cfg);
// reducing pipeline modes (AR / RS / RED), dispatched on (op, kind)
int launch_pipe_reduce(int op, int kind, const PipeArgs &a, const LaunchCfg &cfg);
// data-movement pipeline modes (AG / BC)
int launch_pipe_copy(const PipeArgs &a, const LaunchCfg &cfg);
// one-shot allgather / broadcast (small messages; a.mv = 1 / 2)
int launch_oneshot_mv(const OneShotArgs &a, const LaunchCfg &cfg);
int launch_pack_strided(const void *src, void *dst, size_t nblocks, size_t blk, size_t stride,
                        int unpack, hipStream_t stream, Done done = Done{});
// MPI_Init: one empty kernel per translation unit (loads every code object; timed there)
int launch_touch_all(hipStream_t stream);
// MPI_Init self-test operands and checks (coll/dispatch.hip k_st_fill / k_st_check)
int launch_selftest_fill(uint32_t *p, size_t n, uint32_t seed, int rank, hipStream_t stream);
int launch_selftest_check(const uint32_t *p, size_t n, uint32_t seed, int nranks, int mode, int arg, uint64_t base,
                          uint32_t *bad, hipStream_t stream);
int launch_pack_runs(const void *src, void *dst, size_t count, size_t extent, const int64_t *offs,
                     const int64_t *lens, int nseg, int unpack, hipStream_t stream, Done done = Done{});

}  // namespace mv2
