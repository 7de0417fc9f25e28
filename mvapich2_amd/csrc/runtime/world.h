// world.h — process-wide runtime state for COMM_WORLD on one node.
//
// One process per GPU.  The control plane is a small /dev/shm segment
// (replacing the reference's shmem-coll region, ch3_shmem_coll.c:1365-1455,
// and PMI for the IPC handle exchange); the data plane is device memory:
//   * signal page per rank (hipDeviceMallocUncached, IPC-shared): 64-bit
//     epoch flags [source rank][workgroup]
//   * one-shot arena per rank (uncached, IPC-shared): [parity][source][slot]
//   * user buffers exported on demand through a hipIpc handle cache keyed by
//     allocation id (the reference's cudaipc regcache, ibv_cuda_ipc.c:71-187)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <string>
#include <unordered_map>
#include <vector>

#include "../common.h"
#include "../coll/kernels.h"

namespace mv2 {

constexpr int kShmMaxRanks = 64;

struct BufDesc {
    hipIpcMemHandle_t handle;
    uint64_t buffer_id;
    uint64_t base;
    uint64_t alloc_size;
    uint64_t offset;
    uint64_t seq;
};

struct alignas(64) ShmRank {
    std::atomic<uint64_t> arrive;  // host barrier generation
    char pad0[56];
    int pid;
    int device;
    int pci_bus;
    int pci_device;
    hipIpcMemHandle_t sig_handle;
    hipIpcMemHandle_t arena_handle;
    uint64_t arena_bytes;
    uint64_t slot_bytes;
    BufDesc desc[2];  // per-call published buffers (send, recv)
};

struct ShmSeg {
    std::atomic<uint64_t> magic;
    std::atomic<int> attached;
    int size;
    int pad;
    ShmRank r[kShmMaxRanks];
};

struct Mapping {
    char *ptr;        // mapped base in this process
    uint64_t peer_base;  // allocation base in the peer's address space
    uint64_t alloc_size;
    uint64_t last_use;
};

struct World {
    bool inited = false;
    bool finalized = false;
    int rank = 0, size = 1, local_rank = 0, device = 0;
    int nshare = 1;  // max over ranks of the ranks sharing one GPU (test setups); same on all ranks
    int cus = 256;   // compute units of this GPU
    hipStream_t stream = nullptr;
    std::string shm_name;
    ShmSeg *shm = nullptr;
    uint64_t bar_gen = 0;
    uint64_t seq = 0;

    uint64_t *sig = nullptr;  // my signal page
    SigTable peer_sig{};
    char *arena = nullptr;
    char *peer_arena[kMaxRanks] = {};
    size_t slot_bytes = 0;

    int *h_err = nullptr;     // pinned host error word written by kernels on timeout
    uint64_t timeout_ticks = 0;
    double wall_clock_khz = 100000.0;

    // tuning
    size_t oneshot_max = 256 * 1024;
    int max_grid = 1024;
    int rl_grid = 4096;       // reduce_local grid cap (tools/rl_variants.hip sweep)

    // timing (bench)
    bool timing = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0.0;

    // ipc caches
    std::unordered_map<uint64_t, hipIpcMemHandle_t> own_handles;  // buffer_id -> handle
    std::unordered_map<uint64_t, Mapping> peer_maps[kMaxRanks];    // (peer) buffer_id -> mapping
    uint64_t use_clock = 0;

    // scratch device buffers (host-buffer staging, misalignment, Reduce non-roots)
    void *scratch[3] = {};
    size_t scratch_bytes[3] = {};
};

World &world();
int world_init();
int world_finalize();
void host_barrier();
int ensure_init_for_device();  // singleton-safe lazy device setup (for Reduce_local before Init)
void *get_scratch(int idx, size_t bytes);

}  // namespace mv2
