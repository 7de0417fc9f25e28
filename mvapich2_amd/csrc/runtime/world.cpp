// world.cpp — bootstrap of COMM_WORLD: rank discovery, /dev/shm control
// segment, host barrier, device selection and the IPC-shared signal pages /
// one-shot arenas.  (Replaces MPI_Init's MV2_Read_env_vars + shmem-coll
// init + CUDA IPC region setup: reference init.c:186-300,
// ch3_shmem_coll.c:1365-1455, ibv_cuda_ipc.c:400.)
#include "world.h"
#include "internode.h"

#include <dirent.h>
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

#include "log.h"
#include "orders.h"

namespace mv2 {

static World g_world;
World &world() { return g_world; }

static int env_int(const char *const *names, int dflt) {
    for (int i = 0; names[i]; ++i) {
        const char *v = getenv(names[i]);
        if (v && *v) return atoi(v);
    }
    return dflt;
}

static long env_long(const char *name, long dflt) {
    const char *v = getenv(name);
    return (v && *v) ? atol(v) : dflt;
}

// start time of the parent process (jiffies since boot): with the parent pid
// it names one launch of one launcher (torchrun agent, mv2run, pytest)
static unsigned long long parent_start_time(pid_t ppid) {
    char path[64];
    snprintf(path, sizeof(path), "/proc/%d/stat", (int)ppid);
    FILE *f = fopen(path, "r");
    if (!f) return 0;
    char buf[1024];
    size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = 0;
    const char *p = strrchr(buf, ')');
    if (!p) return 0;
    // fields after ')' start at field 3; starttime is field 22
    int field = 2;
    unsigned long long st = 0;
    for (const char *q = p + 1; *q; ++q) {
        if (*q == ' ') {
            ++field;
            if (field == 22) {
                st = strtoull(q + 1, nullptr, 10);
                break;
            }
        }
    }
    return st;
}

static std::string job_key() {
    const char *j = getenv("MV2AMD_JOBID");
    if (j && *j) return std::string(j);
    pid_t pp = getppid();
    char buf[128];
    const char *port = getenv("MASTER_PORT");
    snprintf(buf, sizeof(buf), "%d_%llu_%s", (int)pp, parent_start_time(pp), port ? port : "0");
    return std::string(buf);
}

static uint64_t mono_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

void beacon(int phase, bool new_call) {
    World &w = g_world;
    if (new_call) ++w.api_calls;
    if (w.size == 1 || !w.shm) return;
    ShmRank &r = w.shm->r[w.rank];
    const uint64_t code = (w.api_calls << 8) | (uint64_t)phase, t = mono_ns();
    r.beacon.store(code, std::memory_order_relaxed);
    r.beacon_ns.store(t, std::memory_order_relaxed);
    const uint32_t k = r.bh_pos.load(std::memory_order_relaxed);
    r.bh_code[k % 16].store(code, std::memory_order_relaxed);
    r.bh_ns[k % 16].store(t, std::memory_order_relaxed);
    r.bh_pos.store(k + 1, std::memory_order_relaxed);
}

void beacon_report(int j, uint64_t now) {
    World &w = g_world;
    if (!w.shm || j < 0 || j >= w.size) return;
    ShmRank &r = w.shm->r[j];
    const uint32_t pos = r.bh_pos.load(std::memory_order_relaxed);
    char line[1024];
    int o = 0;
    for (uint32_t i = pos > 16 ? pos - 16 : 0; i < pos && o < (int)sizeof(line) - 64; ++i) {
        const uint64_t c = r.bh_code[i % 16].load(std::memory_order_relaxed), t = r.bh_ns[i % 16].load(std::memory_order_relaxed);
        o += snprintf(line + o, sizeof(line) - o, " %llu:%d@-%.1fms", (unsigned long long)(c >> 8), (int)(c & 0xff),
                      t && now > t ? (now - t) / 1e6 : 0.0);
    }
    line[o] = 0;
    MV2_ERR("    local rank %d beacon history (call:phase@age):%s", j, line);
}

const char *beacon_name(int phase) {
    switch (phase) {
    case BC_ENTRY: return "entered a call, before its first kernel launch (planning / staging copies)";
    case BC_LAUNCH: return "launching the call's kernel";
    case BC_WAIT: return "waiting for its kernel to complete";
    case BC_DONE: return "between calls (the last one completed)";
    case BC_BARRIER: return "in a host barrier";
    case BC_P2P_WAIT: return "waiting for a point-to-point request";
    case BC_NET: return "on the leaders' inter-node links";
    case BC_SCRATCH: return "growing device scratch (hipFree + hipMalloc)";
    case BC_STAGE: return "staging operands to the device";
    case BC_COPY_OUT: return "copying a result out";
    case BC_LAUNCHED: return "after the kernel launch";
    default: return "not yet in a call";
    }
}

void host_barrier() {
    World &w = g_world;
    if (w.size == 1 || !w.shm) return;
    beacon(BC_BARRIER);
    const uint64_t g = ++w.bar_gen;
    w.shm->r[w.rank].arrive.store(g, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = (double)env_long("MV2AMD_TIMEOUT_S", 120);
    for (int j = 0; j < w.size; ++j) {
        unsigned spins = 0;
        while (w.shm->r[j].arrive.load(std::memory_order_acquire) < g) {
            if (++spins > 2000) {
                sched_yield();
                if ((spins & 0xfff) == 0) {
                    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    if (el > limit) MV2_FATAL("host barrier timed out after %.0f s waiting for rank %d", el, j);
                }
            }
        }
    }
}

namespace {
struct HostWin {
    char *p = nullptr;
    size_t cap = 0;
    int fd = -1;
    bool pinned = false;  // own window: registered with HIP, so device copies to and from it are DMA
};
HostWin g_own_win;
HostWin g_peer_win[kMaxRanks];
std::string window_name(int r) { return g_world.shm_name + ".ux" + std::to_string(r); }
}  // namespace

char *host_window(size_t bytes) {
    World &w = g_world;
    if (!w.shm || w.size <= 1) return nullptr;
    HostWin &o = g_own_win;
    if (bytes <= o.cap) return o.p;
    if (o.fd < 0 && (o.fd = shm_open(window_name(w.rank).c_str(), O_CREAT | O_RDWR, 0600)) < 0) {
        MV2_DEBUG("host window: shm_open failed");
        return nullptr;
    }
    const size_t page = 1 << 21;
    size_t want = std::max(bytes, 2 * o.cap);
    want = (want + page - 1) / page * page;
    if (posix_fallocate(o.fd, 0, (off_t)want) != 0) {  // a small /dev/shm: the exact size, or nothing
        want = (bytes + 4095) / 4096 * 4096;
        if (posix_fallocate(o.fd, 0, (off_t)want) != 0) {
            MV2_DEBUG("host window: /dev/shm has no room for %zu bytes", bytes);
            return nullptr;
        }
    }
    if (o.p) {
        if (o.pinned) hipHostUnregister(o.p);
        munmap(o.p, o.cap);
    }
    void *q = mmap(nullptr, want, PROT_READ | PROT_WRITE, MAP_SHARED, o.fd, 0);
    if (q == MAP_FAILED) {
        o.p = nullptr;
        o.cap = 0;
        o.pinned = false;
        return nullptr;
    }
    o.p = (char *)q;
    o.cap = want;
    o.pinned = hipHostRegister(o.p, o.cap, hipHostRegisterDefault) == hipSuccess;
    if (!o.pinned) (void)hipGetLastError();  // still usable, through staged copies
    return o.p;
}

const char *host_peer_window(int r, size_t bytes) {
    if (r < 0 || r >= kMaxRanks) return nullptr;
    HostWin &v = g_peer_win[r];
    if (v.p && v.cap >= bytes) return v.p;
    const int fd = shm_open(window_name(r).c_str(), O_RDONLY, 0);
    if (fd < 0) return nullptr;
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < bytes) {
        close(fd);
        return nullptr;
    }
    if (v.p) munmap(v.p, v.cap);
    void *q = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
    close(fd);
    if (q == MAP_FAILED) {
        v.p = nullptr;
        v.cap = 0;
        return nullptr;
    }
    v.p = (char *)q;
    v.cap = (size_t)st.st_size;
    return v.p;
}

bool host_window_vote(bool ok) {
    World &w = g_world;
    if (w.size == 1 || !w.shm) return ok;
    host_barrier();  // every window reserved (or not)
    w.shm->r[w.rank].window_ok = ok ? 1 : 0;
    host_barrier();
    bool all = true;
    for (int j = 0; j < w.size; ++j) all = all && w.shm->r[j].window_ok;
    host_barrier();  // every vote read before the next vote overwrites it
    return all;
}

static void host_windows_release() {
    World &w = g_world;
    for (HostWin &v : g_peer_win) {
        if (v.p) munmap(v.p, v.cap);
        v = HostWin{};
    }
    if (g_own_win.p) {
        if (g_own_win.pinned) hipHostUnregister(g_own_win.p);
        munmap(g_own_win.p, g_own_win.cap);
    }
    if (g_own_win.fd >= 0) {
        close(g_own_win.fd);
        shm_unlink(window_name(w.rank).c_str());
    }
    g_own_win = HostWin{};
}

// The most ranks (and node leaders) a flat algorithm runs as per-element programs across nodes:
// kMaxRanks, or fewer with MV2AMD_MN_PROG_MAX (tests: the message schedules of jobs above 8 ranks
// on jobs small enough to share one GPU without oversubscribing its hardware scheduler, DESIGN.md
// §5 "Ranks per GPU")
int mn_prog_max() {
    static const int m = [] {
        const long v = env_long("MV2AMD_MN_PROG_MAX", kMaxRanks);
        return (int)(v < 1 ? 1 : v > kMaxRanks ? kMaxRanks : v);
    }();
    return m;
}

void *get_scratch(int idx, size_t bytes) {
    World &w = g_world;
    if (w.scratch_bytes[idx] >= bytes && w.scratch[idx]) return w.scratch[idx];
    beacon(BC_SCRATCH);
    if (w.scratch[idx]) {
        // a collective abandoned with a receive still arriving may target this block: it is left
        // allocated (never reused) rather than freed under the transport (runtime/p2p.cpp)
        if (!coll_context_poisoned()) {
            hipStreamSynchronize(w.stream);
            hipFree(w.scratch[idx]);
        }
        w.scratch[idx] = nullptr;
        w.scratch_bytes[idx] = 0;
    }
    size_t sz = bytes < 4096 ? 4096 : bytes;
    ++w.call_allocs;
    if (hipMalloc(&w.scratch[idx], sz) != hipSuccess) return nullptr;
    w.scratch_bytes[idx] = sz;
    return w.scratch[idx];
}

// ---------------------------------------------------------------------------
// Device temporaries of MPI calls: derived-type staging (MPI_Bcast / MPI_Allgather of a
// non-contiguous type, MPI_Pack / MPI_Unpack between host and device memory) and the packed
// payload of a non-contiguous MPI_Isend / MPI_Irecv, which lives until the request completes, so
// several can be held at once.  Blocks are kept for reuse instead of a hipMalloc / hipFree per
// call (hipFree synchronises the whole device, serialising the call against every stream); the
// reference keeps its device staging the same way (device_stage_alloc, ch3_shmem_coll.c:3433).
// Sizes round up to a power of two (>= 64 KiB) so that nearby sizes share blocks; a failed
// allocation first returns the idle blocks to HIP and tries once more.
// ---------------------------------------------------------------------------
namespace {
struct PoolBlock {
    void *p;
    size_t cap;
    bool used;
};
std::vector<PoolBlock> g_pool;
}  // namespace

// MV2AMD_POOL=0: a hipMalloc per pool_get and a hipFree per pool_put (round 4's behaviour, kept
// as a knob for the before / after measurement)
static bool pool_on() {
    static const bool on = env_long("MV2AMD_POOL", 1) != 0;
    return on;
}

void *pool_get(size_t bytes) {
    World &w = g_world;
    if (!pool_on()) {
        void *p = nullptr;
        ++w.call_allocs;
        return hipMalloc(&p, bytes ? bytes : 1) == hipSuccess ? p : nullptr;
    }
    PoolBlock *best = nullptr;
    for (PoolBlock &b : g_pool)
        if (!b.used && b.cap >= bytes && (!best || b.cap < best->cap)) best = &b;
    if (best) {
        best->used = true;
        return best->p;
    }
    size_t cap = (size_t)64 << 10;
    while (cap < bytes) cap <<= 1;
    beacon(BC_SCRATCH);
    ++w.call_allocs;
    void *p = nullptr;
    if (hipMalloc(&p, cap) != hipSuccess) {
        (void)hipGetLastError();
        if (w.stream) hipStreamSynchronize(w.stream);
        for (size_t i = 0; i < g_pool.size();)
            if (!g_pool[i].used) {
                hipFree(g_pool[i].p);
                g_pool.erase(g_pool.begin() + (long)i);
            } else {
                ++i;
            }
        if (hipMalloc(&p, cap) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
    }
    g_pool.push_back(PoolBlock{p, cap, true});
    return p;
}

// Idle blocks kept for reuse are capped (MV2AMD_POOL_IDLE_MAX bytes, default 256 MiB): above it
// pool_put returns the largest idle blocks to HIP, so one large unexpected message or derived-type
// staging does not pin its power-of-two block of HBM for the rest of the job.
static size_t pool_idle_max() {
    static const size_t m = (size_t)env_long("MV2AMD_POOL_IDLE_MAX", 256L << 20);
    return m;
}

void pool_put(void *p) {
    if (!pool_on()) {
        if (p) hipFree(p);
        return;
    }
    size_t idle = 0;
    for (PoolBlock &b : g_pool) {
        if (b.p == p) b.used = false;
        if (!b.used) idle += b.cap;
    }
    while (idle > pool_idle_max()) {
        size_t big = g_pool.size();
        for (size_t i = 0; i < g_pool.size(); ++i)
            if (!g_pool[i].used && (big == g_pool.size() || g_pool[i].cap > g_pool[big].cap)) big = i;
        if (big == g_pool.size()) break;
        idle -= g_pool[big].cap;
        hipFree(g_pool[big].p);
        g_pool.erase(g_pool.begin() + (long)big);
        ++g_world.pool_trims;
    }
}

static void pool_release_all() {
    for (PoolBlock &b : g_pool) hipFree(b.p);
    g_pool.clear();
}

// GPUs this process can see, counted without initialising HIP: the KFD topology's GPU nodes,
// narrowed by a visibility list if one is set (every entry counts as one device)
static int gpus_visible_before_hip() {
    int n = 0;
    for (int i = 0; i < 256; ++i) {
        char path[96];
        snprintf(path, sizeof(path), "/sys/class/kfd/kfd/topology/nodes/%d/gpu_id", i);
        FILE *f = fopen(path, "r");
        if (!f) break;
        long id = 0;
        if (fscanf(f, "%ld", &id) == 1 && id != 0) ++n;
        fclose(f);
    }
    for (const char *v : {"ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"}) {
        const char *e = getenv(v);
        if (!e || !*e) continue;
        int k = 1;
        for (const char *c = e; *c; ++c) k += *c == ',';
        if (n == 0 || k < n) n = k;
    }
    return n;
}

// Several ranks on one GPU (tests, the one-GPU box, mv2run --share-gpu): every collective
// kernel needs its peers' kernels resident at the same time, and with HIP's default 4 hardware
// queues per process five ranks' queues starve each other — one rank's kernel was not dispatched
// for 30 s while the others' kernels spun (profiles/r04f_queue_starvation.txt; 3 ms with 2 queues
// per process).  So before HIP starts, a process that will share its GPU lowers GPU_MAX_HW_QUEUES
// to 2 (unset, or set higher — the one-GPU box exports HIP's default 4); MV2AMD_HW_QUEUES=0 leaves
// it alone, =k asks for k.  One rank per GPU is not touched.  Returns the value set, or 0.
static int limit_hw_queues_if_shared(int local_size) {
    const long want = env_long("MV2AMD_HW_QUEUES", 2);
    const long have = env_long("GPU_MAX_HW_QUEUES", 0);
    if (want <= 0 || (have > 0 && have <= want)) return 0;
    const int ndev = gpus_visible_before_hip();
    const bool shared = env_long("MV2AMD_NSHARE", 1) > 1 || (getenv("MV2AMD_DEVICE") && local_size > 1) ||
                        (ndev > 0 && local_size > ndev);
    if (!shared) return 0;
    char v[24];
    snprintf(v, sizeof(v), "%ld", want);
    setenv("GPU_MAX_HW_QUEUES", v, 1);
    return (int)want;
}

// Is HIP already running in this process (a host framework or an earlier call touched the GPU
// first)?  The ROCm runtime opens /dev/kfd when it starts, so an open descriptor on it says so;
// GPU_MAX_HW_QUEUES is read once at that start, so setting it later has no effect.
static bool hip_already_running() {
    DIR *d = opendir("/proc/self/fd");
    if (!d) return false;
    bool found = false;
    char path[300], target[64];
    while (struct dirent *e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        snprintf(path, sizeof(path), "/proc/self/fd/%s", e->d_name);
        const ssize_t k = readlink(path, target, sizeof(target) - 1);
        if (k <= 0) continue;
        target[k] = 0;
        if (!strcmp(target, "/dev/kfd")) {
            found = true;
            break;
        }
    }
    closedir(d);
    return found;
}

static int env_local_size() {
    const char *lsn[] = {"MV2_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "OMPI_COMM_WORLD_LOCAL_SIZE", "LOCAL_WORLD_SIZE",
                         nullptr};
    const char *sn[] = {"MV2_COMM_WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "WORLD_SIZE", nullptr};
    return env_int(lsn, env_int(sn, 1));
}

// limit_hw_queues_if_shared before this library's own HIP start-up: records what was set (> 0),
// or -k when k queues were wanted but HIP was already running (the setting came too late)
static void apply_hw_queue_limit(int local_size) {
    World &w = g_world;
    if (w.stream || w.hw_queues_set) return;
    const bool late = hip_already_running();
    const int q = limit_hw_queues_if_shared(local_size);
    w.hw_queues_set = late && q > 0 ? -q : q;
    // kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1): the command processor then reads
    // them from HBM instead of over PCIe.  Measured on the 8-byte MPI_Reduce_local, whose call is
    // mostly launch and dispatch: 8.60 -> 8.02 us and 8.11 -> 7.32 us on two boxes (profiles/r06e).
    // Like GPU_MAX_HW_QUEUES it is read once when HIP starts; a value set by the user wins, and
    // MV2AMD_DEV_KERNARG=0 leaves HIP's default.
    if (!late && !getenv("HIP_FORCE_DEV_KERNARG") && env_long("MV2AMD_DEV_KERNARG", 1) != 0)
        setenv("HIP_FORCE_DEV_KERNARG", "1", 0);
}

static int setup_device_common() {
    World &w = g_world;
    const auto t_hip = std::chrono::steady_clock::now();
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        MV2_ERR("no HIP device visible: this library runs its reduction path on MI355X only");
        return E_OTHER;
    }
    const char *dn[] = {"MV2AMD_DEVICE", nullptr};
    w.device = env_int(dn, w.local_rank % ndev);
    if (hipSetDevice(w.device) != hipSuccess) return E_OTHER;
    w.sync_mode = (int)env_long("MV2AMD_SYNC", w.sync_mode);
    // blocking stream: orders after legacy null-stream work (buffer readiness)
    if (hipStreamCreate(&w.stream) != hipSuccess) return E_OTHER;
    if (hipHostMalloc((void **)&w.h_err, kErrWords * sizeof(int), hipHostMallocDefault) != hipSuccess) return E_OTHER;
    memset(w.h_err, 0, kErrWords * sizeof(int));
    if (hipMalloc((void **)&w.done_ctr, kDoneBytes) != hipSuccess || hipMemset(w.done_ctr, 0, kDoneBytes) != hipSuccess ||
        hipHostMalloc((void **)&w.done_flag, 64, hipHostMallocDefault) != hipSuccess) {
        w.done_ctr = nullptr;
        w.done_flag = nullptr;
        w.sync_mode = 1;
    } else {
        memset(w.done_flag, 0, 64);
        hipDeviceSynchronize();
    }
    hipDeviceGetAttribute(&w.cus, hipDeviceAttributeMultiprocessorCount, w.device);
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, w.device) == hipSuccess && khz > 0)
        w.wall_clock_khz = khz;
    w.timeout_ticks = (uint64_t)(env_long("MV2AMD_TIMEOUT_S", 120) * w.wall_clock_khz * 1000.0);
    w.oneshot_max = (size_t)env_long("MV2AMD_ONESHOT_MAX", (long)w.oneshot_max);
    w.max_grid = (int)std::min<long>(env_long("MV2AMD_MAX_GRID", w.max_grid), kDoneMaxGrid);
    w.pipe_grid = (int)env_long("MV2AMD_PIPE_GRID", w.pipe_grid);
    w.pipe_sub = (size_t)env_long("MV2AMD_PIPE_SUB", (long)w.pipe_sub);
    w.pipe_rnt = env_long("MV2AMD_PIPE_RNT", w.pipe_rnt) != 0;  // stores into peers' arenas: non-temporal / plain
    w.light_release = (int)env_long("MV2AMD_LIGHT_RELEASE", w.light_release);
    w.rl_grid = (int)std::min<long>(env_long("MV2AMD_RL_GRID", w.rl_grid), kDoneMaxGrid);
    w.rl_tiny_max = (size_t)std::max(0L, env_long("MV2AMD_RL_TINY_MAX", (long)w.rl_tiny_max));
    knobs_reload();  // MV2_* algorithm-selection knobs (orders.cpp)
    hipEventCreate(&w.ev0);
    hipEventCreate(&w.ev1);
    w.hip_init_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_hip).count();
    // every code object of the library loaded here, timed (MV2AMD_PRELOAD_KERNELS=0: left to HIP's
    // deferred loading at each unit's first launch)
    if (env_long("MV2AMD_PRELOAD_KERNELS", 1) != 0) {
        const auto t_load = std::chrono::steady_clock::now();
        if (launch_touch_all(w.stream) != 0 || hipStreamSynchronize(w.stream) != hipSuccess) {
            MV2_ERR("loading the library's gfx950 code objects failed: %s", hipGetErrorString(hipGetLastError()));
            return E_OTHER;
        }
        w.code_load_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_load).count();
    }
    return 0;
}

int ensure_init_for_device() {
    World &w = g_world;
    if (w.stream) return 0;
    if (!getenv("MV2AMD_CONTROL_PLANE_ONLY")) apply_hw_queue_limit(env_local_size());
    return setup_device_common();
}


// ---------------------------------------------------------------------------
// Intra-node topology levels (orders.h Topo): this rank's cluster id per level as the reference
// derives them at MPI_Init (init.c:255-271 -> smpi_identify_my_numa_id, hwloc_bind.c:2252-2298,
// then smpi_identify_my_sock_id :2180-2250), from this process's CPU binding (the reference reads
// its own, hwloc_get_proc_cpubind) and the sysfs view of the NUMA nodes and packages.  The
// reference binds its ranks itself first (MV2_ENABLE_AFFINITY, bunch policy); this library does
// not bind, so unbound ranks all intersect the first NUMA node and form one group (one level).
// MV2AMD_TOPO="c0,c1,...[;d0,d1,...]" gives every local rank's ids per level instead.
// ---------------------------------------------------------------------------
static bool read_cpulist(const char *path, std::vector<int> &cpus) {
    FILE *f = fopen(path, "r");
    if (!f) return false;
    char buf[4096];
    const bool ok = fgets(buf, sizeof(buf), f) != nullptr;
    fclose(f);
    if (!ok) return false;
    for (char *p = buf; *p && *p != '\n';) {
        char *e = nullptr;
        const long a = strtol(p, &e, 10);
        if (e == p) break;
        long b = a;
        p = e;
        if (*p == '-') {
            b = strtol(p + 1, &e, 10);
            p = e;
        }
        for (long c = a; c <= b; ++c) cpus.push_back((int)c);
        if (*p == ',') ++p;
    }
    return true;
}

static int my_topology(int *color, int max_levels) {
    int n = 0;
    cpu_set_t mine;
    CPU_ZERO(&mine);
    if (sched_getaffinity(0, sizeof(mine), &mine) != 0) return 0;
    std::vector<int> online;
    if (!read_cpulist("/sys/devices/system/cpu/online", online)) return 0;
    auto intersects = [&](const std::vector<int> &cs) {
        for (int c : cs)
            if (c < CPU_SETSIZE && CPU_ISSET(c, &mine)) return true;
        return false;
    };
    // NUMA nodes in index order (hwloc logical order = OS order here)
    std::vector<int> nodes;
    read_cpulist("/sys/devices/system/node/online", nodes);
    std::vector<std::vector<int>> node_cpus(nodes.size());
    int my_numa = -1;
    for (size_t i = 0; i < nodes.size(); ++i) {
        char path[128];
        snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", nodes[i]);
        read_cpulist(path, node_cpus[i]);
        if (my_numa < 0 && intersects(node_cpus[i])) my_numa = (int)i;
    }
    if (nodes.size() > 1 && n < max_levels) color[n++] = my_numa;
    // packages: sorted physical ids; the first one this binding intersects
    std::vector<int> pkg_ids, pkg_of(online.size(), -1);
    for (size_t k = 0; k < online.size(); ++k) {
        char path[128];
        snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/topology/physical_package_id", online[k]);
        FILE *f = fopen(path, "r");
        int id = -1;
        if (f) {
            if (fscanf(f, "%d", &id) != 1) id = -1;
            fclose(f);
        }
        pkg_of[k] = id;
        if (id >= 0 && std::find(pkg_ids.begin(), pkg_ids.end(), id) == pkg_ids.end()) pkg_ids.push_back(id);
    }
    std::sort(pkg_ids.begin(), pkg_ids.end());
    int my_sock = -1;
    std::vector<int> sock_cpus;
    for (size_t i = 0; i < pkg_ids.size() && my_sock < 0; ++i) {
        std::vector<int> cs;
        for (size_t k = 0; k < online.size(); ++k)
            if (pkg_of[k] == pkg_ids[i]) cs.push_back(online[k]);
        if (intersects(cs)) {
            my_sock = (int)i;
            sock_cpus = cs;
        }
    }
    if (pkg_ids.size() > 1) {
        // the NUMA node of the last level (0 without one) inside this socket: no socket level
        const int numa_id = n >= 1 ? color[n - 1] : 0;
        bool inside = false;
        if (numa_id >= 0 && (size_t)numa_id < node_cpus.size()) {
            inside = true;
            for (int c : node_cpus[numa_id])
                if (std::find(sock_cpus.begin(), sock_cpus.end(), c) == sock_cpus.end()) inside = false;
        }
        if (!inside && n < max_levels) color[n++] = my_sock;
    }
    return n;
}

// MV2AMD_TOPO override: level l's ids are the l-th ';'-separated list, one id per local rank
static int topo_override(int rank, int *color, int max_levels) {
    const char *v = getenv("MV2AMD_TOPO");
    if (!v || !*v) return -1;
    int n = 0;
    for (const char *p = v; *p && n < max_levels;) {
        int idx = 0, val = 0;
        bool found = false;
        while (*p && *p != ';') {
            char *e = nullptr;
            const long x = strtol(p, &e, 10);
            if (e == p) break;
            if (idx == rank) {
                val = (int)x;
                found = true;
            }
            ++idx;
            p = e;
            if (*p == ',') ++p;
        }
        color[n++] = found ? val : 0;
        while (*p && *p != ';') ++p;
        if (*p == ';') ++p;
    }
    return n;
}

int world_init() {
    World &w = g_world;
    if (w.inited) return 0;
    const auto t_init = std::chrono::steady_clock::now();
    auto ms_since = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    const char *rn[] = {"MV2_COMM_WORLD_RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK", "RANK", nullptr};
    const char *sn[] = {"MV2_COMM_WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "WORLD_SIZE", nullptr};
    const char *ln[] = {"MV2_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "LOCAL_RANK", nullptr};
    const char *lsn[] = {"MV2_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "OMPI_COMM_WORLD_LOCAL_SIZE", "LOCAL_WORLD_SIZE", nullptr};
    w.rank = env_int(rn, 0);
    w.size = env_int(sn, 1);
    w.local_rank = env_int(ln, w.rank);
    const int lsize = env_int(lsn, w.size);
    if (w.size < 1 || w.rank < 0 || w.rank >= w.size) {
        MV2_ERR("invalid rank/size from environment: rank=%d size=%d", w.rank, w.size);
        return E_OTHER;
    }
    w.grank = w.rank;
    w.gsize = w.size;
    if (lsize != w.size) {
        // several nodes: this process's world below is its node (rank = local rank); the
        // leaders (local rank 0) add the inter-node links (internode.cpp).  Ranks must be
        // numbered node-major with the same count per node (the reference's is_blocked /
        // is_uniform communicators, create_2level_comm.c)
        if (lsize < 1 || w.size % lsize != 0 || w.local_rank < 0 || w.local_rank >= lsize ||
            w.rank != (w.rank / lsize) * lsize + w.local_rank) {
            MV2_ERR("multi-node launch needs node-major ranks and the same ranks per node "
                    "(rank %d, local rank %d, local size %d, size %d)", w.rank, w.local_rank, lsize, w.size);
            return E_UNSUPPORTED;
        }
        w.nnodes = w.size / lsize;
        w.node = w.rank / lsize;
        w.rank = w.local_rank;
        w.size = lsize;
    }
    if (w.size > kShmMaxRanks) {
        MV2_ERR("world size %d exceeds %d", w.size, kShmMaxRanks);
        return E_UNSUPPORTED;
    }
    // MV2AMD_CONTROL_PLANE_ONLY=1: bootstrap the shm control plane without a
    // GPU (CPU tests of rank discovery / barriers).  Every data-path entry
    // point still requires the device and fails loudly without it.
    const char *cpo = getenv("MV2AMD_CONTROL_PLANE_ONLY");
    const bool control_only = cpo && *cpo == '1';
    if (!w.stream && !control_only) {
        apply_hw_queue_limit(w.size);
        int rc = setup_device_common();
        if (rc) return rc;
    }

    if (w.size > 1) {
        w.shm_name = "/mv2amd." + job_key() + (w.nnodes > 1 ? ".n" + std::to_string(w.node) : std::string());
        int fd = shm_open(w.shm_name.c_str(), O_CREAT | O_RDWR, 0600);
        if (fd < 0) {
            MV2_ERR("shm_open(%s) failed", w.shm_name.c_str());
            return E_OTHER;
        }
        if (ftruncate(fd, sizeof(ShmSeg)) != 0) {
            close(fd);
            return E_OTHER;
        }
        void *p = mmap(nullptr, sizeof(ShmSeg), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) return E_OTHER;
        w.shm = (ShmSeg *)p;
        ShmRank &me = w.shm->r[w.rank];
        me.pid = getpid();
        me.device = w.device;
        if (!control_only) {
            hipDeviceGetAttribute(&me.pci_domain, hipDeviceAttributePciDomainId, w.device);
            hipDeviceGetAttribute(&me.pci_bus, hipDeviceAttributePciBusId, w.device);
            hipDeviceGetAttribute(&me.pci_device, hipDeviceAttributePciDeviceId, w.device);
        }
        memcpy(&me.knobs, &knobs(), sizeof(Knobs));
        me.topo_nlevels = topo_override(w.rank, me.topo_color, kTopoLevels);
        if (me.topo_nlevels < 0) me.topo_nlevels = my_topology(me.topo_color, kTopoLevels);
        w.shm->attached.fetch_add(1);
        host_barrier();  // everyone attached and published pid/device/knobs
        // the algorithm choice (and with it the kernels' flag pairing) must agree on every
        // rank: a rank started with different MV2_* selection knobs would hang the job
        for (int j = 0; j < w.size; ++j)
            if (memcmp(&w.shm->r[j].knobs, &knobs(), sizeof(Knobs)) != 0) {
                MV2_ERR("MV2_* collective selection knobs differ between rank %d and rank %d", w.rank, j);
                return E_OTHER;
            }

        // topology levels (orders.h Topo): every rank's cluster ids, levels past a rank's
        // own count read 0 (mv2_intra_node_cluster_at_level is zero-initialised)
        {
            Topo t{};
            for (int j = 0; j < w.size && j < kMaxRanks; ++j) {
                const ShmRank &q = w.shm->r[j];
                if (q.topo_nlevels > t.nlevels) t.nlevels = q.topo_nlevels;
                for (int l = 0; l < kTopoLevels; ++l) t.color[l][j] = l < q.topo_nlevels ? q.topo_color[l] : 0;
            }
            topo_set(t);
        }

        // ranks sharing one GPU (tests run several ranks on one device): the
        // maximum over all GPUs, so every rank derives the same kernel grids
        w.nshare = 1;
        for (int i = 0; i < w.size; ++i) {
            int c = 0;
            for (int j = 0; j < w.size; ++j)
                if (w.shm->r[j].pci_domain == w.shm->r[i].pci_domain && w.shm->r[j].pci_bus == w.shm->r[i].pci_bus &&
                    w.shm->r[j].pci_device == w.shm->r[i].pci_device)
                    ++c;
            if (c > w.nshare) w.nshare = c;
        }
        // emulated nodes on one GPU (tests, mv2run --nodes --share-gpu): the GPU is shared with
        // the other nodes' ranks too, which this node's segment cannot see
        const long ns = env_long("MV2AMD_NSHARE", 0);
        if (ns > w.nshare) w.nshare = (int)ns;
        // Above 8 processes on one GPU (its hardware scheduler's concurrent processes, KFD's VMIDs)
        // the emulated-node soaks returned wrong bytes: a rank's own send buffer held another rank's
        // previous operand before the call (profiles/r05ar, r05at; r06b-r06d: 3-21 wrong calls of 400
        // at 12 = 3 x 4, 35-86 with the copy engines off).  The cause is not found (DESIGN.md "Ranks
        // per GPU": the same traffic without this library stays exact at 9-16 processes, and the
        // workgroups' XCD placement held), so such a job is refused here, on every rank, instead of
        // returning wrong sums later.  MV2AMD_UNSAFE_OVERSUBSCRIBE=1 lets it run for diagnosis only,
        // with a warning on every rank.
        if (w.nshare > kHwsProcs && !control_only) {
            if (env_long("MV2AMD_UNSAFE_OVERSUBSCRIBE", 0) != 1) {
                MV2_ERR("%d processes share one GPU, more than the %d its hardware scheduler runs at once: "
                        "device collectives between them are not supported (DESIGN.md \"Ranks per GPU\"); "
                        "run at most %d ranks per GPU",
                        w.nshare, kHwsProcs, kHwsProcs);
                host_barrier();  // every rank of the node has read the segment; remove it
                shm_unlink(w.shm_name.c_str());
                return E_UNSUPPORTED;
            }
            fprintf(stderr,
                    "[mv2amd rank %d] warning: %d processes share one GPU (MV2AMD_UNSAFE_OVERSUBSCRIBE=1): "
                    "results of device collectives may be wrong above %d\n",
                    log_rank(), w.nshare, kHwsProcs);
        }

        if (w.size <= kMaxRanks && !control_only) {
            // signal page + one-shot arena, IPC-exported
            const size_t sig_bytes = (size_t)kMaxRanks * kMaxBlocks * sizeof(uint64_t);
            if (hipExtMallocWithFlags((void **)&w.sig, sig_bytes, hipDeviceMallocUncached) != hipSuccess) {
                MV2_ERR("hipExtMallocWithFlags(uncached) for the signal page failed");
                return E_NO_MEM;
            }
            hipMemset(w.sig, 0, sig_bytes);
            w.slot_bytes = (w.oneshot_max + 4095) & ~(size_t)4095;
            // when MPI_Init will time the one-shot / pipelined crossover on this node's links (one
            // rank per GPU, or MV2AMD_PIPE_AUTOTUNE=1) and no limit is set, the slots hold up to
            // 1 MiB so that the probe can find a crossover above the 256 KiB default: on xGMI a
            // one-shot call of 512 KiB - 1 MiB moves (n-1) x size per rank in one flag exchange
            // against the pipelined kernel's two (coll.cpp oneshot_autotune)
            {
                const long at = env_long("MV2AMD_PIPE_AUTOTUNE", -1);
                const bool tunes = at == 1 || (at < 0 && w.nshare == 1);
                if (tunes && !getenv("MV2AMD_ONESHOT_MAX") && !getenv("MV2AMD_PIPE_GRID") && !getenv("MV2AMD_PIPE_SUB"))
                    w.slot_bytes = std::max(w.slot_bytes, (size_t)1 << 20);
            }
            const size_t arena_bytes = 2 * (size_t)kMaxRanks * w.slot_bytes;
            if (hipExtMallocWithFlags((void **)&w.arena, arena_bytes, hipDeviceMallocUncached) != hipSuccess) {
                MV2_ERR("hipExtMallocWithFlags(uncached) for the one-shot arena failed");
                return E_NO_MEM;
            }
            if (hipExtMallocWithFlags((void **)&w.p2p, kP2PArena, hipDeviceMallocUncached) != hipSuccess) {
                MV2_ERR("hipExtMallocWithFlags(uncached) for the point-to-point arena failed");
                return E_NO_MEM;
            }
            if (hipExtMallocWithFlags((void **)&w.pipe_rs, kPipeRegion, hipDeviceMallocUncached) != hipSuccess ||
                hipExtMallocWithFlags((void **)&w.pipe_ag, kPipeRegion, hipDeviceMallocUncached) != hipSuccess) {
                MV2_ERR("hipExtMallocWithFlags(uncached) for the pipeline arenas (2 x %zu MiB) failed",
                        kPipeRegion >> 20);
                return E_NO_MEM;
            }
            // graph lane (MV2AMD_GRAPH_LANE=0 leaves it out): the same layout again, for
            // collectives captured into HIP graphs, whose sequence numbers live on the device
            w.graph_lane = env_long("MV2AMD_GRAPH_LANE", 1) != 0;
            if (w.graph_lane &&
                (hipExtMallocWithFlags((void **)&w.g_sig, sig_bytes, hipDeviceMallocUncached) != hipSuccess ||
                 hipExtMallocWithFlags((void **)&w.g_arena, arena_bytes, hipDeviceMallocUncached) != hipSuccess ||
                 hipExtMallocWithFlags((void **)&w.g_rs, kPipeRegion, hipDeviceMallocUncached) != hipSuccess ||
                 hipExtMallocWithFlags((void **)&w.g_ag, kPipeRegion, hipDeviceMallocUncached) != hipSuccess ||
                 hipExtMallocWithFlags((void **)&w.dseq, sizeof(DevSeq), hipDeviceMallocUncached) != hipSuccess)) {
                MV2_ERR("graph lane: device allocation failed");
                return E_NO_MEM;
            }
            if (w.graph_lane) {
                w.g_pool_bytes = (size_t)env_long("MV2AMD_GRAPH_POOL", 4L << 20);
                if (hipMalloc((void **)&w.g_pool, w.g_pool_bytes) != hipSuccess) return E_NO_MEM;
                hipMemset(w.g_sig, 0, sig_bytes);
                hipMemset(w.dseq, 0, sizeof(DevSeq));
                if (hipIpcGetMemHandle(&me.g_sig_handle, w.g_sig) != hipSuccess ||
                    hipIpcGetMemHandle(&me.g_arena_handle, w.g_arena) != hipSuccess ||
                    hipIpcGetMemHandle(&me.g_rs_handle, w.g_rs) != hipSuccess ||
                    hipIpcGetMemHandle(&me.g_ag_handle, w.g_ag) != hipSuccess) {
                    MV2_ERR("hipIpcGetMemHandle failed for the graph lane");
                    return E_OTHER;
                }
            }
            me.graph_lane = w.graph_lane ? 1 : 0;
            hipDeviceSynchronize();
            if (hipIpcGetMemHandle(&me.sig_handle, w.sig) != hipSuccess ||
                hipIpcGetMemHandle(&me.arena_handle, w.arena) != hipSuccess ||
                hipIpcGetMemHandle(&me.pipe_rs_handle, w.pipe_rs) != hipSuccess ||
                hipIpcGetMemHandle(&me.pipe_ag_handle, w.pipe_ag) != hipSuccess ||
                hipIpcGetMemHandle(&me.p2p_handle, w.p2p) != hipSuccess) {
                MV2_ERR("hipIpcGetMemHandle failed for the signal page / arenas");
                return E_OTHER;
            }
            me.arena_bytes = arena_bytes;
            me.slot_bytes = w.slot_bytes;
            host_barrier();
            for (int j = 0; j < w.size; ++j) {
                if (j == w.rank) {
                    w.peer_sig.p[j] = w.sig;
                    w.peer_arena[j] = w.arena;
                    w.peer_rs.p[j] = w.pipe_rs;
                    w.peer_ag.p[j] = w.pipe_ag;
                    w.peer_p2p[j] = w.p2p;
                    w.g_peer_sig.p[j] = w.g_sig;
                    w.g_peer_arena[j] = w.g_arena;
                    w.g_peer_rs.p[j] = w.g_rs;
                    w.g_peer_ag.p[j] = w.g_ag;
                    continue;
                }
                if (w.shm->r[j].graph_lane != (w.graph_lane ? 1 : 0)) {
                    MV2_ERR("MV2AMD_GRAPH_LANE differs between ranks");
                    return E_OTHER;
                }
                if (w.graph_lane) {
                    void *q[4] = {};
                    if (hipIpcOpenMemHandle(&q[0], w.shm->r[j].g_sig_handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
                        hipIpcOpenMemHandle(&q[1], w.shm->r[j].g_arena_handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
                        hipIpcOpenMemHandle(&q[2], w.shm->r[j].g_rs_handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
                        hipIpcOpenMemHandle(&q[3], w.shm->r[j].g_ag_handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                        MV2_ERR("hipIpcOpenMemHandle failed for rank %d's graph lane", j);
                        return E_OTHER;
                    }
                    w.g_peer_sig.p[j] = (uint64_t *)q[0];
                    w.g_peer_arena[j] = (char *)q[1];
                    w.g_peer_rs.p[j] = (char *)q[2];
                    w.g_peer_ag.p[j] = (char *)q[3];
                }
                if (w.shm->r[j].slot_bytes != w.slot_bytes) {
                    MV2_ERR("MV2AMD_ONESHOT_MAX differs between ranks");
                    return E_OTHER;
                }
                void *ps = nullptr, *pa = nullptr, *pr = nullptr, *pg = nullptr, *pp = nullptr;
                if (hipIpcOpenMemHandle(&ps, w.shm->r[j].sig_handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
                    hipIpcOpenMemHandle(&pa, w.shm->r[j].arena_handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
                    hipIpcOpenMemHandle(&pr, w.shm->r[j].pipe_rs_handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
                    hipIpcOpenMemHandle(&pg, w.shm->r[j].pipe_ag_handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
                    hipIpcOpenMemHandle(&pp, w.shm->r[j].p2p_handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                    MV2_ERR("hipIpcOpenMemHandle failed for rank %d (peer access over xGMI?)", j);
                    return E_OTHER;
                }
                w.peer_sig.p[j] = (uint64_t *)ps;
                w.peer_arena[j] = (char *)pa;
                w.peer_rs.p[j] = (char *)pr;
                w.peer_ag.p[j] = (char *)pg;
                w.peer_p2p[j] = (char *)pp;
            }
            host_barrier();
        }
    }
    if (w.size == 1 && !control_only) {
        void *p = mmap(nullptr, sizeof(ShmSeg), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) return E_NO_MEM;
        w.shm = (ShmSeg *)p;
        if (hipExtMallocWithFlags((void **)&w.p2p, kP2PArena, hipDeviceMallocUncached) != hipSuccess) {
            MV2_ERR("hipExtMallocWithFlags(uncached) for the point-to-point arena failed");
            return E_NO_MEM;
        }
        w.peer_p2p[0] = w.p2p;
    }
    w.inited = true;
    if (w.size > 1 && w.size <= kMaxRanks && !control_only && env_long("MV2AMD_SELFTEST", 1) != 0) {
        const auto t_st = std::chrono::steady_clock::now();
        int rc = coll_selftest();
        w.selftest_ms = ms_since(t_st);
        const auto t_tune = std::chrono::steady_clock::now();
        if (!rc) rc = pipe_autotune();
        w.tune_ms = ms_since(t_tune);
        if (rc) {
            w.inited = false;
            return rc;
        }
    }
    if (w.nnodes > 1) {
        int rc = w.rank == 0 ? net_init() : 0;
        if (w.shm && w.rank == 0) w.shm->net_rc.store(rc);
        host_barrier();  // the node's leader is linked to every other node (or failed: all ranks fail)
        if (w.shm) rc = w.shm->net_rc.load();
        if (rc) {
            if (w.rank != 0) MV2_ERR("the node leader's inter-node bootstrap failed");
            w.inited = false;
            return rc;
        }
        if ((rc = mesh_setup())) {  // every rank linked to the ranks of the other nodes (p2p)
            w.inited = false;
            return rc;
        }
    }
    w.init_ms = ms_since(t_init);
    // one line on the job's rank 0 (stderr) naming what MPI_Init decided for this node's
    // device collectives, so a run's log explains itself even without its result line
    // (MV2AMD_INIT_REPORT=0: silent; =1: also for a single-rank job)
    const long rep = env_long("MV2AMD_INIT_REPORT", -1);
    if (w.grank == 0 && (rep > 0 || (rep < 0 && w.gsize > 1))) {
        const bool ran = w.size > 1 && w.size <= kMaxRanks && env_long("MV2AMD_SELFTEST", 1) != 0;
        int g256 = 0;
        size_t t256 = 0;
        pipe_tiling_for(((size_t)256 << 20) / (size_t)w.size, &g256, &t256);  // a 256 MiB allreduce's segment
        char qnote[160] = "";
        if (w.hw_queues_set > 0)
            snprintf(qnote, sizeof(qnote), "; GPU shared: GPU_MAX_HW_QUEUES lowered to %d", w.hw_queues_set);
        else if (w.hw_queues_set < 0)
            snprintf(qnote, sizeof(qnote), "; GPU shared, but HIP was already running: GPU_MAX_HW_QUEUES=%d came too "
                     "late (set it before the process starts HIP)", -w.hw_queues_set);
        fprintf(stderr,
                "[mv2amd] MPI_Init: %d ranks (%d per node, %d node%s, %d per GPU); self-test %s%d calls checked%s; "
                "tiling %s, %s stores (256 MiB allreduce: %d workgroups x %zu KiB per round); one-shot up to %zu KiB; "
                "init %.1f ms (HIP start %.1f, code objects %.1f, self-test %.1f, autotune %.1f)%s\n",
                w.gsize, w.size, w.nnodes, w.nnodes > 1 ? "s" : "", w.nshare, !ran ? "not run (" : "passed (",
                w.selftest_calls, !ran ? ")" : w.light_release ? "), light release" : "), full system-scope release",
                w.pipe_tuned ? "autotuned" : "default", w.pipe_rnt ? "non-temporal" : "plain", g256, t256 >> 10,
                w.oneshot_max >> 10, w.init_ms, w.hip_init_ms, w.code_load_ms, w.selftest_ms, w.tune_ms, qnote);
        fflush(stderr);
    }
    MV2_DEBUG("init rank %d/%d local %d device %d nshare %d (node %d of %d): %.1f ms (self-test %.1f, autotune %.1f)",
              w.grank, w.gsize, w.rank, w.device, w.nshare, w.node, w.nnodes, w.init_ms, w.selftest_ms, w.tune_ms);
    return 0;
}

int global_barrier() {
    World &w = world();
    host_barrier();
    int rc = 0;
    if (w.nnodes > 1 && w.rank == 0) rc = net_barrier();
    host_barrier();
    return rc;
}

int world_finalize() {
    World &w = g_world;
    if (!w.inited || w.finalized) return 0;
    if (w.stream) hipStreamSynchronize(w.stream);
    host_prof_report();
    aql_finalize();
    if (w.nnodes > 1) {
        global_barrier();
        net_finalize();  // the rank mesh on every rank, the leaders' links on the leaders
    }
    if (w.size > 1 && w.shm) {
        host_barrier();
        host_windows_release();
        for (int j = 0; j < kMaxRanks; ++j) {
            if (j != w.rank && j < w.size && w.size <= kMaxRanks) {
                if (w.peer_sig.p[j]) hipIpcCloseMemHandle(w.peer_sig.p[j]);
                if (w.peer_arena[j]) hipIpcCloseMemHandle(w.peer_arena[j]);
                if (w.peer_rs.p[j]) hipIpcCloseMemHandle(w.peer_rs.p[j]);
                if (w.peer_ag.p[j]) hipIpcCloseMemHandle(w.peer_ag.p[j]);
                if (w.peer_p2p[j]) hipIpcCloseMemHandle(w.peer_p2p[j]);
                if (w.graph_lane) {
                    if (w.g_peer_sig.p[j]) hipIpcCloseMemHandle(w.g_peer_sig.p[j]);
                    if (w.g_peer_arena[j]) hipIpcCloseMemHandle(w.g_peer_arena[j]);
                    if (w.g_peer_rs.p[j]) hipIpcCloseMemHandle(w.g_peer_rs.p[j]);
                    if (w.g_peer_ag.p[j]) hipIpcCloseMemHandle(w.g_peer_ag.p[j]);
                }
            }
        }
        host_barrier();  // nobody maps our pages any more
        if (w.rank == 0) shm_unlink(w.shm_name.c_str());
        munmap(w.shm, sizeof(ShmSeg));
        w.shm = nullptr;
    }
    for (int i = 0; i < (int)(sizeof(w.scratch) / sizeof(w.scratch[0])); ++i)
        if (w.scratch[i]) hipFree(w.scratch[i]);
    pool_release_all();
    if (w.sig) hipFree(w.sig);
    if (w.arena) hipFree(w.arena);
    if (w.pipe_rs) hipFree(w.pipe_rs);
    if (w.pipe_ag) hipFree(w.pipe_ag);
    if (w.p2p) hipFree(w.p2p);
    for (void *p : {(void *)w.g_sig, (void *)w.g_arena, (void *)w.g_rs, (void *)w.g_ag, (void *)w.dseq, (void *)w.g_pool})
        if (p) hipFree(p);
    w.finalized = true;
    return 0;
}

}  // namespace mv2
