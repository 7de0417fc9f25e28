// world.h — process-wide runtime state for COMM_WORLD on one node.
//
// One process per GPU.  The control plane is a small /dev/shm segment
// (replacing the reference's shmem-coll region, ch3_shmem_coll.c:1365-1455,
// and PMI for the IPC handle exchange); the data plane is device memory:
//   * signal page per rank (hipDeviceMallocUncached, IPC-shared): 64-bit
//     epoch flags [source rank][workgroup]
//   * one-shot arena per rank (uncached, IPC-shared): [parity][source][slot]
//   * pipeline arenas per rank (uncached, IPC-shared): RS and AG regions of
//     [parity][source][kPipeSlot] (coll/pipe.h)
// User buffers are never exported: peers only ever store into these
// library-owned arenas, so an application may hipFree a buffer right after
// a call (the reference's cudaipc regcache, ibv_cuda_ipc.c:71-187, is not
// needed and its stale-mapping hazard does not exist).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <string>
#include <vector>

#include "../common.h"
#include "../coll/kernels.h"
#include "orders.h"

namespace mv2 {

constexpr int kShmMaxRanks = 64;

// Point-to-point channels (runtime/p2p.cpp): per ordered pair (src -> dst) a
// FIFO of kP2PSlots chunk records in the control segment and kP2PSlots data
// slots of kP2PChunk bytes in dst's IPC-exported, uncached P2P arena.
constexpr int kP2PSlots = 4;
constexpr size_t kP2PChunk = (size_t)8 << 20;
constexpr size_t kP2PArena = (size_t)kMaxRanks * kP2PSlots * kP2PChunk;  // 256 MiB per rank

struct P2PRec {
    uint64_t msg;    // sender's message sequence number
    int32_t tag;
    int32_t pad;
    uint64_t total;  // message bytes
    uint64_t off;    // byte offset of this chunk
    uint64_t len;    // bytes in this chunk (0 only for an empty message)
};

struct alignas(64) P2PChan {
    std::atomic<uint64_t> tail;  // chunk records published by the sender
    char pad0[56];
    std::atomic<uint64_t> head;  // chunk records consumed by the receiver (slot freed)
    char pad1[56];
    P2PRec rec[kP2PSlots];
};

constexpr int kTuneMax = 16;  // pipe_autotune candidates

struct alignas(64) ShmRank {
    std::atomic<uint64_t> arrive;  // host barrier generation
    char pad0[56];
    int pid;
    int device;
    int pci_domain;  // with bus and device: the GPU's identity (segments may reuse bus numbers)
    int pci_bus;
    int pci_device;
    hipIpcMemHandle_t sig_handle;
    hipIpcMemHandle_t arena_handle;
    uint64_t arena_bytes;
    uint64_t slot_bytes;
    hipIpcMemHandle_t pipe_rs_handle;
    hipIpcMemHandle_t pipe_ag_handle;
    hipIpcMemHandle_t p2p_handle;
    hipIpcMemHandle_t g_sig_handle, g_arena_handle, g_rs_handle, g_ag_handle;  // graph lane
    int graph_lane;   // 1: this rank allocated the graph lane
    int selftest_ok;  // coll_selftest verdict of this rank (agreed through host_barrier)
    int window_ok;    // host_window_vote: this rank's window and its partners' views are in place
    double tune_us[kTuneMax];  // pipe_autotune: this rank's time per candidate tiling
    Knobs knobs;      // MV2_* selection knobs as this rank parsed them (must agree)
    int topo_nlevels;               // this rank's topology levels (world.cpp my_topology)
    int topo_color[kTopoLevels];    // its cluster id per level
    int mesh_port;                  // this rank's rank-mesh listener (internode.cpp mesh_setup)
    // where this rank's host is (world.cpp beacon): (API call number << 8) | Beacon phase, and
    // when it got there; a peer whose device wait runs out prints every late rank's beacon
    std::atomic<uint64_t> beacon;
    std::atomic<uint64_t> beacon_ns;
    std::atomic<uint64_t> bh_code[16], bh_ns[16];  // the last 16 beacons (history ring)
    std::atomic<uint32_t> bh_pos;
};

constexpr int kHwsProcs = 8;  // processes one GPU's hardware scheduler runs at once (KFD's VMIDs)
constexpr int kMeshMaxRanks = 64;  // jobs up to this many ranks get the rank mesh (p2p across nodes)

struct ShmSeg {
    std::atomic<uint64_t> magic;
    std::atomic<int> attached;
    int size;
    std::atomic<int> tune_stop;  // pipe_autotune: rank 0 ends the probe once its time budget is spent
    std::atomic<int> net_rc;     // the leader's inter-node bootstrap result, for the node's other ranks
    ShmRank r[kShmMaxRanks];
    P2PChan chan[kMaxRanks][kMaxRanks];  // [src][dst]
    int mesh_port[kMeshMaxRanks];        // every rank's rank-mesh listener (the leader fills it in)
    char node_ip[kMeshMaxRanks][48];     // every node's address
};

struct World {
    bool inited = false;
    bool finalized = false;
    int rank = 0, size = 1, local_rank = 0, device = 0;  // this node's world (rank = local rank)
    // the job: global rank / size; nodes of `size` ranks each, ranks numbered node-major
    // (rank = node * size + local rank); nnodes > 1 adds the leader transport (internode.cpp)
    int grank = 0, gsize = 1, node = 0, nnodes = 1;
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
    // pipelined-collective arenas (coll/pipe.h): RS and AG regions, kPipeRegion bytes each
    char *pipe_rs = nullptr, *pipe_ag = nullptr;
    PeerTableW peer_rs{}, peer_ag{};
    uint64_t epoch = 0;       // last flag epoch used (identical on every rank)
    uint64_t round = 0;       // pipeline rounds issued (slot parity)
    uint64_t os_calls = 0;    // one-shot calls issued (arena parity)
    // the last launches that took flag epochs (a timeout report names the one that waited)
    struct EpochRec {
        uint64_t call, lo, hi;
        int user_stream;
    };
    EpochRec epoch_log[8] = {};
    unsigned epoch_pos = 0;

    // graph lane (HIP graph capture of stream-ordered allreduce, coll.cpp): its own signal page,
    // one-shot arena and pipeline arenas, with the sequence numbers kept on the device (DevSeq)
    bool graph_lane = false;
    bool graph = false;  // the current call is being captured into a graph
    uint64_t *g_sig = nullptr;
    SigTable g_peer_sig{};
    char *g_arena = nullptr;
    char *g_peer_arena[kMaxRanks] = {};
    char *g_rs = nullptr, *g_ag = nullptr;
    PeerTableW g_peer_rs{}, g_peer_ag{};
    DevSeq *dseq = nullptr;
    char *g_pool = nullptr;        // staging pieces of captured calls (never reused)
    size_t g_pool_bytes = 0, g_pool_used = 0;

    // point-to-point (runtime/p2p.cpp)
    char *p2p = nullptr;                  // my P2P arena: [src][slot] chunks
    char *peer_p2p[kMaxRanks] = {};       // rank j's P2P arena (mapped; entry me = mine)
    hipStream_t p2p_stream = nullptr;     // chunk copies (separate from the collectives' stream)

    int *h_err = nullptr;     // pinned host error word written by kernels on timeout
    uint64_t timeout_ticks = 0;
    double wall_clock_khz = 100000.0;

    // tuning
    size_t oneshot_max = 256 * 1024;
    int max_grid = 1024;
    int pipe_grid = kPipeMaxGrid;                 // pipelined collectives: workgroups (<= kPipeMaxGrid)
    size_t pipe_sub = kPipeMaxSub;                // bytes per workgroup per segment per round
    int light_release = 1;                        // signal without L2 writeback (arena data is uncached)
    int pipe_tuned = 0;                           // 1: pipe_grid / pipe_sub chosen by pipe_autotune
    int pipe_rnt = 1;                             // stores into peers' arenas: 1 non-temporal, 0 plain
    int tune_rnt[kTuneMax] = {};
    int os_tune_n = 0;                            // one-shot threshold probe: sizes 32 KiB << i
    double os_tune_us[kTuneMax / 2][2] = {};      // [size][one-shot, pipelined], max over ranks
    int tune_n = 0;                               // candidates timed by pipe_autotune
    int tune_grid[kTuneMax] = {};
    size_t tune_sub[kTuneMax] = {};
    double tune_us[kTuneMax] = {};                // max over ranks per candidate
    double init_ms = 0, selftest_ms = 0, tune_ms = 0;  // MPI_Init wall time and its self-test / autotune parts
    // HIP start-up (first HIP call through stream creation) and the first kernel launch of this
    // library (loads its gfx950 code object: HIP defers that to the first launch)
    double hip_init_ms = 0, code_load_ms = 0;
    int selftest_calls = 0;  // collective calls MPI_Init's self-test checked (all ranks, every element)
    // device allocations made inside MPI calls (scratch growth: hipMalloc, each paired with a
    // hipFree that synchronises the device); stays flat once the scratch caches are warm
    uint64_t call_allocs = 0;
    uint64_t pool_trims = 0;  // idle pool blocks returned to HIP above MV2AMD_POOL_IDLE_MAX (world.cpp pool_put)
    // completion-word events (coll.cpp wait_done), reported by mv2h_get_info and both bench lines:
    // the stream was consulted (the word unseen 200 us after the launch); the word was seen only
    // after the stream reported the kernel finished; the kernel had ended without raising it; the
    // kernel raised it marked "groups split over XCDs" (device_util.h block_done), so the host
    // completed the call with a stream synchronisation
    uint64_t done_queried = 0, done_late = 0, done_missed = 0, done_xcd_split = 0;
    uint64_t split_seen = 0;  // last done_flag[1] (split call's seq) already settled
    size_t uop_in_bytes = 0, uop_area_bytes = 0;  // last host-evaluated reduction: operand bytes received, area
    // host-evaluated reductions, cumulative ns per phase (mpi/user_coll.cpp UopPhase): staging the
    // operands (device pack + exchange), fetching them to the host (D2H + unpack), evaluating (uop
    // calls + result pack), delivering (H2D + results' exchange + device unpack)
    uint64_t uop_ns[4] = {0, 0, 0, 0};
    uint64_t api_calls = 0;  // library calls entered (the beacon's call number)
    int hw_queues_set = 0;   // GPU_MAX_HW_QUEUES this library set before HIP started (ranks sharing a GPU)
    int rl_grid = 1 << 20;    // reduce_local grid cap (default: one tile per workgroup, tools/rl_variants.hip)
    size_t rl_tiny_max = 1024;  // reduce_local operands up to this many bytes: one-wave kernel (MV2AMD_RL_TINY_MAX)
    uint64_t aql_calls = 0;     // reduce_local calls dispatched straight into the HSA queue (runtime/aql.cpp)
    bool stream_hip_busy = true;  // HIP may still count work on `stream` as running (set by every launch there)
    int sync_mode = 0;        // completion wait: 0 kernel-written completion word, 1 hipStreamSynchronize only
    uint32_t *done_ctr = nullptr;   // device: 9 arrival counters of the completion word (Done)
    uint64_t *done_flag = nullptr;  // pinned host: last completed call's sequence number
    uint64_t done_seq = 0;          // last sequence number armed
    uint64_t pending = 0;           // seq the current call waits for (0: stream sync)
    bool defer = false;             // nonblocking initiation: finish() leaves the wait to a ticket
    bool enqueue = false;           // stream-ordered call (mv2h_*_enqueue): launch on the caller's stream, no wait
    hipStream_t last_st = nullptr;  // stream of the last library launch (cross-stream ordering, pick_stream)
    hipEvent_t sw_ev = nullptr;     // recorded on last_st when a call switches streams
    uint64_t deferred = 0;          // ticket of the last deferred call (0: completed at initiation)

    // timing (bench)
    bool timing = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0.0;

    // scratch device buffers (host-buffer staging, misalignment, Reduce non-roots)
    void *scratch[7] = {};  // 5: multi-node Reduce_scatter's result, 6: multi-node ring's node operands
    size_t scratch_bytes[7] = {};
};

World &world();
int world_init();
int world_finalize();
// runtime/aql.cpp: small MPI_Reduce_local dispatched straight into an HSA queue (1 done, 0 not
// taken, < 0 an MPI error class); the kernels it found; its queue torn down at MPI_Finalize
int aql_reduce_local(int op, int kind, const void *in, void *io, size_t count, size_t esize);
int aql_kernels();
int aql_acquire_scope();  // the HSA-queue Reduce_local's acquire scope: 1 agent, 2 system, -1 path off
long aql_skips(int which);  // 0: library words pending, 1: null stream busy
void aql_finalize();
void host_barrier();
// Host shared-memory windows between the ranks of a node, for host-evaluated reductions that
// exchange partial results the way the reference's point-to-point algorithms do: this rank's
// window (grown on demand, backed by /dev/shm space reserved up front so a full tmpfs is an
// error here and not a SIGBUS later), and a read-only view of a node peer's window of at least
// `bytes` (nullptr when the peer's window is smaller or absent).  Released by world_finalize.
char *host_window(size_t bytes);
const char *host_peer_window(int rank, size_t bytes);
// Every rank of the node votes `ok`; returns true on every rank iff all voted true (three host
// barriers: windows reserved before the vote, votes read by everyone before the next one).
bool host_window_vote(bool ok);
// beacon phases (ShmRank::beacon)
enum Beacon { BC_ENTRY = 1, BC_LAUNCH = 2, BC_WAIT = 3, BC_DONE = 4, BC_BARRIER = 5, BC_P2P_WAIT = 6, BC_NET = 7,
              BC_SCRATCH = 8, BC_STAGE = 9, BC_COPY_OUT = 10, BC_LAUNCHED = 11 };
void beacon_report(int j, uint64_t now);  // print local rank j's beacon history (stderr)
void beacon(int phase, bool new_call = false);
const char *beacon_name(int phase);
int global_barrier();  // node barrier, leaders' barrier across nodes, node barrier
int ensure_init_for_device();  // singleton-safe lazy device setup (for Reduce_local before Init)
void *get_scratch(int idx, size_t bytes);
// device temporaries of MPI calls, kept for reuse (world.cpp): a block of >= bytes, or nullptr
void *pool_get(size_t bytes);
void pool_put(void *p);  // back to the pool (the device work using it has completed)
bool coll_context_poisoned();  // runtime/p2p.cpp: an abandoned collective request is still in flight
unsigned long long p2p_unexpected_matched();  // runtime/p2p.cpp: unexpected messages later taken by a receive
// runtime/coll.cpp: across nodes, the most ranks (and node leaders) a flat algorithm runs as
// per-element programs; above it, its message schedule (MV2AMD_MN_PROG_MAX, default kMaxRanks)
int mn_prog_max();
int coll_selftest();  // coll.cpp: init-time check of the cross-GPU publish protocol
void pipe_tiling_for(size_t seg_bytes, int *grid, size_t *tsub);  // coll.cpp: a segment's grid and bytes per round
int pipe_autotune();  // coll.cpp: init-time choice of the pipelined kernels' tiling
void host_prof_report();  // coll.cpp: MV2AMD_HOST_PROFILE summary
// The library's own messages on the node's point-to-point channels (the steps of the multi-node
// collectives) carry tags below kCollTagBase: the collective context of MPICH's comm (context_id +
// MPID_CONTEXT_INTRA_COLL), so no application receive, MPI_ANY_TAG included, can match them.
constexpr int kCollTagBase = -0x100;
int p2p_isend(const void *buf, size_t bytes, int dest, int tag, unsigned long long *req);  // runtime/p2p.cpp
int p2p_irecv(void *buf, size_t cap, int source, int tag, unsigned long long *req);
// a collective's request given up after an error: an unmatched receive is withdrawn; one whose data
// is still arriving (or a send still in flight) poisons the collective context, so every later
// library collective fails instead of matching stale messages (runtime/p2p.cpp)
void p2p_abandon(unsigned long long req);

}  // namespace mv2
