// kernels.h — host-side launch interface of the HIP kernels (C++ only, internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../device_util.h"

namespace mv2 {

struct TreeParams {
    int linear;      // 1: LINEAR order, 0: BUTTERFLY
    int pof2, rem, lg;
    int owner_fixed; // >= 0: fixed owner newrank; -1: reduce-scatter block owner
    size_t rs_blk;   // elements per reduce-scatter block (count / pof2)
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
};

struct TwoShotArgs {
    PeerTable src;    // every rank's sendbuf (mapped into this process)
    PeerTable agsrc;  // every rank's recvbuf (mapped)
    char *recv;
    SigTable sig_peer;
    uint64_t *sig_own;
    size_t count, nvec;
    int n, me;
    TreeParams tp;
    uint64_t epoch;   // uses epoch, epoch+1, epoch+2
    int *err;
    uint64_t timeout;
};

struct RsArgs {
    PeerTable src;    // every rank's sendbuf (mapped)
    char *dst;        // my result region base (aligned like src + off)
    SigTable sig_peer;
    uint64_t *sig_own;
    size_t off, cnt;  // my block: elements [off, off+cnt)
    int n, me;
    TreeParams tp;
    uint64_t epoch;   // epoch, epoch+1
    int *err;
    uint64_t timeout;
};

struct GatherArgs {
    PeerTable src;    // per source rank: base to read (mapped), nullptr = skip
    char *dst;        // my destination base
    size_t dst_off[kMaxRanks];  // byte offset in dst for source j
    size_t bytes;     // bytes per source
    SigTable sig_peer;
    uint64_t *sig_own;
    int n, me;
    uint64_t epoch;   // epoch, epoch+1
    int *err;
    uint64_t timeout;
};

struct LaunchCfg {
    int grid;
    int unroll;
    hipStream_t stream;
    int cus = 256;    // compute units of the device
    int nshare = 1;   // max ranks sharing one GPU (same on every rank)
};

// vectors per thread per tile of the two-shot kernel: fewer sources -> more
// vectors, so every thread keeps >= 8 16-byte loads in flight
inline int twoshot_unroll(int n) { return n <= 3 ? 4 : 2; }

// Workgroups that are guaranteed co-resident for a kernel (the per-workgroup
// cross-GPU flags need block b of every rank running together).  The
// occupancy API can over-report by one block per CU (MI355X_MICROARCH.md,
// Residency), so one block per CU is held back.
inline int resident_grid(const void *kernel, const LaunchCfg &cfg) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, kThreads, 0) != hipSuccess || nb < 1) nb = 1;
    nb = nb > 1 ? nb - 1 : 1;
    int cap = nb * cfg.cus / (cfg.nshare > 0 ? cfg.nshare : 1);
    return cap < 1 ? 1 : cap;
}

// all return an MPI error class (0 = launched)
int launch_reduce_local(int op, int kind, const void *in, void *inout, size_t count, size_t esize,
                        const LaunchCfg &cfg);
int launch_reduce_n(int op, int kind, const void *const *srcs, int n, void *dst, size_t count,
                    size_t esize, const TreeParams &tp, const LaunchCfg &cfg);
int launch_oneshot(int op, int kind, const OneShotArgs &a, size_t esize, const LaunchCfg &cfg);
int launch_twoshot(int op, int kind, const TwoShotArgs &a, size_t esize, const LaunchCfg &cfg);
int launch_rs(int op, int kind, const RsArgs &a, size_t esize, const LaunchCfg &cfg);
int launch_gather(const GatherArgs &a, const LaunchCfg &cfg);
int launch_pack_strided(const void *src, void *dst, size_t nblocks, size_t blk, size_t stride,
                        int unpack, hipStream_t stream);

}  // namespace mv2
