// aql.cpp — the 8-byte path of MPI_Reduce_local: the one-wave kernel dispatched straight into an
// HSA queue of this library's own, without hipLaunchKernel.
//
// An 8-byte MPI_Reduce_local on device buffers is all launch and dispatch: the kernel itself is one
// wave.  Measured on MI355X (tools/diag/rl_lat.cpp, profiles/r06e): hipLaunchKernel costs 2.3-3.0 us
// of host time per launch, and the floor of "launch a one-wave kernel, see its pinned host word"
// through HIP is 6.0-6.4 us, against 8.5 us for the library call in round 5.  Writing the AQL
// packet ourselves costs a few hundred nanoseconds of host time.
//
// The kernel objects are HIP's own: k_reduce_local_tiny<R<op, kind>> from this library's code
// objects, which MPI_Init loads (world.cpp, code-object preload), found through the AMD loader
// extension (every executable of the process, its kernel symbols for this GPU) and keyed by the
// (op, kind) in the mangled name.  The queue is created once on the HSA agent of this rank's HIP
// device.  A packet carries an agent-scope acquire and no release (see Aql::acquire); the kernel
// releases its result and raises the call's completion word (device_util.h contract) and the host
// spins on it, as for a HIP launch.
//
// Ordering: the HIP path runs on the library's blocking stream, ordered after the legacy null
// stream's work.  This queue is outside HIP's ordering, so the fast path is taken only when the
// library's own work is done (every completion word it armed has been raised) and the null stream
// is idle (hipStreamQuery); otherwise, and whenever the
// path is unavailable (MV2AMD_AQL=0, ranks sharing a GPU, a symbol or the queue missing), the call
// takes the HIP launch.  A word that does not arrive within 10 s is an error and turns the path off.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>

#include "../common.h"
#include "../device_util.h"
#include "log.h"
#include "world.h"

namespace mv2 {
namespace {

struct KObj {
    uint64_t object = 0;
    uint32_t private_bytes = 0, group_bytes = 0;
};

struct Aql {
    int state = 0;  // 0 untried, 1 ready, -1 unavailable
    hsa_agent_t agent{};
    hsa_queue_t *queue = nullptr;
    char *kernarg = nullptr;  // kRing slots of kSlot bytes (fine-grained system memory)
    KObj k[OP_COUNT][K_COUNT];
    int kernels = 0;
    uint64_t skip_lib = 0, skip_null = 0;  // calls that took the HIP launch: library words pending / null stream busy
    bool hsa_ref = false;  // aql_init's hsa_init reference, released by aql_finalize
    // the packet's fences: an agent-scope acquire (this CU's caches invalidated before the kernel
    // reads its operands) and no release -- the kernel releases its result at system scope itself
    // before raising the word.  The operands' producers completed before the call through HIP
    // (stream or device synchronisation, or the library's own words), whose completion releases
    // them from every XCD's L2; tools/diag/stale_probe.hip rewrote an operand 3,000 times by a copy
    // engine and 3,000 times by a kernel on a HIP stream between two kernels of such a queue that
    // read it on every XCD, and saw no stale word even with no acquire at all (profiles/r06/r06p).
    // A system-scope acquire costs ~0.9-1.5 us more per call (DESIGN.md §6 *8-byte latency*).
    // That probe cannot cover a writer on another GPU (over xGMI into this GPU's memory, which does
    // not pass this GPU's L2s), so a job with other ranks keeps the system scope (aql_init).
    // MV2AMD_AQL_ACQUIRE / _RELEASE: 0 none, 1 agent, 2 system.
    int acquire = HSA_FENCE_SCOPE_AGENT, release = HSA_FENCE_SCOPE_NONE;
    int acquire_set = -1;  // MV2AMD_AQL_ACQUIRE, else agent for a one-rank job and system otherwise
    int stream_checks = 1;  // MV2AMD_AQL_STREAM_CHECKS=0: measurement only (drops the null-stream ordering)
    std::atomic<int> queue_error{0};
};
Aql g_aql;
constexpr int kRing = 64, kSlot = 64;

// explicit arguments of k_reduce_local_tiny (kernels_impl.h): in, io, count, flag, seq
struct TinyArgs {
    const void *in;
    void *io;
    uint32_t count, pad;
    uint64_t *flag;
    uint64_t seq;
};
static_assert(sizeof(TinyArgs) == 40, "k_reduce_local_tiny's kernarg segment is 40 bytes");

struct AgentFind {
    uint32_t bdfid;
    uint32_t domain;
    hsa_agent_t agent;
    bool found;
};

hsa_status_t find_agent(hsa_agent_t a, void *data) {
    AgentFind *f = (AgentFind *)data;
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
        return HSA_STATUS_SUCCESS;
    uint32_t bdf = 0, dom = 0;
    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
    if (bdf == f->bdfid && dom == f->domain) {
        f->agent = a;
        f->found = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

hsa_status_t find_kernarg_region(hsa_region_t r, void *data) {
    hsa_region_segment_t seg;
    if (hsa_region_get_info(r, HSA_REGION_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS || seg != HSA_REGION_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &flags);
    if (flags & HSA_REGION_GLOBAL_FLAG_KERNARG) {
        *(hsa_region_t *)data = r;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

// "..._ZN3mv219k_reduce_local_tinyINS_1RILi<op>ELi<kind>EvEEEE..." -> op, kind
bool parse_tiny(const char *name, int *op, int *kind) {
    const char *p = strstr(name, "k_reduce_local_tiny");
    if (!p || !(p = strstr(p, "RILi"))) return false;
    char *end = nullptr;
    const long o = strtol(p + 4, &end, 10);
    if (!end || strncmp(end, "ELi", 3) != 0) return false;
    const long k = strtol(end + 3, &end, 10);
    if (!end || *end != 'E' || o < 0 || o >= OP_COUNT || k < 0 || k >= K_COUNT) return false;
    *op = (int)o;
    *kind = (int)k;
    return true;
}

hsa_status_t take_symbol(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void *) {
    hsa_symbol_kind_t kind;
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
        kind != HSA_SYMBOL_KIND_KERNEL)
        return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len) != HSA_STATUS_SUCCESS || len == 0 ||
        len > 4096)
        return HSA_STATUS_SUCCESS;
    char name[4100];
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, name) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    name[len] = 0;
    int op, k;
    if (!parse_tiny(name, &op, &k)) return HSA_STATUS_SUCCESS;
    uint32_t kargs = 0;
    KObj o;
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &o.object) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kargs) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &o.private_bytes) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &o.group_bytes) !=
            HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    // only the layout this file writes (no hidden arguments): anything else keeps the HIP launch
    if (kargs != sizeof(TinyArgs) || !o.object) return HSA_STATUS_SUCCESS;
    if (!g_aql.k[op][k].object) ++g_aql.kernels;
    g_aql.k[op][k] = o;
    return HSA_STATUS_SUCCESS;
}

hsa_status_t take_executable(hsa_executable_t e, void *) {
    hsa_executable_iterate_agent_symbols(e, g_aql.agent, take_symbol, nullptr);
    return HSA_STATUS_SUCCESS;
}

void queue_error_cb(hsa_status_t status, hsa_queue_t *, void *) {
    g_aql.queue_error.store((int)status);
}

uint64_t now_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

int aql_init() {
    World &w = world();
    g_aql.state = -1;
    const char *on = getenv("MV2AMD_AQL");
    if ((on && *on == '0') || w.nshare > 1 || !w.done_flag) return -1;
    if (hsa_init() != HSA_STATUS_SUCCESS) return -1;  // reference-counted: HIP's runtime is already up
    g_aql.hsa_ref = true;
    int bus = 0, dev = 0, dom = 0;
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, w.device) != hipSuccess ||
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, w.device) != hipSuccess ||
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, w.device) != hipSuccess)
        return -1;
    AgentFind f{(uint32_t)((bus << 8) | (dev << 3)), (uint32_t)dom, {}, false};
    hsa_iterate_agents(find_agent, &f);
    if (!f.found) {
        MV2_DEBUG("aql: no HSA agent for PCI %04x:%02x:%02x", dom, bus, dev);
        return -1;
    }
    g_aql.agent = f.agent;
    hsa_ven_amd_loader_1_03_pfn_t ldr{};
    if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(ldr), &ldr) != HSA_STATUS_SUCCESS ||
        !ldr.hsa_ven_amd_loader_iterate_executables)
        return -1;
    ldr.hsa_ven_amd_loader_iterate_executables(take_executable, nullptr);
    if (g_aql.kernels == 0) {
        MV2_DEBUG("aql: no k_reduce_local_tiny kernel objects found");
        return -1;
    }
    hsa_region_t kr{};
    hsa_agent_iterate_regions(f.agent, find_kernarg_region, &kr);
    if (!kr.handle || hsa_memory_allocate(kr, (size_t)kRing * kSlot, (void **)&g_aql.kernarg) != HSA_STATUS_SUCCESS)
        return -1;
    memset(g_aql.kernarg, 0, (size_t)kRing * kSlot);
    uint32_t qmin = 0, qmax = 0;
    hsa_agent_get_info(f.agent, HSA_AGENT_INFO_QUEUE_MIN_SIZE, &qmin);
    hsa_agent_get_info(f.agent, HSA_AGENT_INFO_QUEUE_MAX_SIZE, &qmax);
    uint32_t qsize = kRing;
    while (qsize < qmin) qsize <<= 1;
    if ((qmax && qsize > qmax) ||
        hsa_queue_create(f.agent, qsize, HSA_QUEUE_TYPE_SINGLE, queue_error_cb, nullptr, UINT32_MAX, UINT32_MAX,
                         &g_aql.queue) != HSA_STATUS_SUCCESS) {
        hsa_memory_free(g_aql.kernarg);
        g_aql.kernarg = nullptr;
        return -1;
    }
    if (const char *e = getenv("MV2AMD_AQL_ACQUIRE")) g_aql.acquire_set = atoi(e) & 3;
    if (const char *e = getenv("MV2AMD_AQL_RELEASE")) g_aql.release = atoi(e) & 3;
    if (const char *e = getenv("MV2AMD_AQL_STREAM_CHECKS")) g_aql.stream_checks = atoi(e) != 0;
    g_aql.state = 1;
    MV2_DEBUG("aql: %d k_reduce_local_tiny kernels, queue of %u packets", g_aql.kernels, g_aql.queue->size);
    return 0;
}

}  // namespace

// 1: the call was dispatched and has completed (the word arrived); 0: not taken (the caller
// launches through HIP); < 0: an MPI error class
// MV2AMD_HOST_PROFILE: entry -> doorbell and doorbell -> word, printed at MPI_Finalize
static uint64_t g_prof_calls, g_prof_pre_ns, g_prof_wait_ns;

int aql_reduce_local(int op, int kind, const void *in, void *io, size_t count, size_t esize) {
    const uint64_t t_entry = now_ns();
    World &w = world();
    if (g_aql.state == 0) aql_init();
    if (g_aql.state != 1 || op < 0 || op >= OP_COUNT || kind < 0 || kind >= K_COUNT) return 0;
    const KObj &ko = g_aql.k[op][kind];
    if (!ko.object || count == 0 || count * esize > w.rl_tiny_max || count > 0xffffffffu) return 0;
    if (w.sync_mode || w.enqueue || w.graph || w.timing) return 0;
    // the HIP path's ordering: every word this library armed has been raised (its calls' work is
    // done -- HIP's own view of the stream lags the word by the kernel's end and its completion
    // signal, so hipStreamQuery(w.stream) would still say "busy" right after a call), and nothing is
    // pending on the legacy null stream
    if (__atomic_load_n(w.done_flag, __ATOMIC_ACQUIRE) < w.done_seq) {
        ++g_aql.skip_lib;
        return 0;
    }
    // HIP's view of the library's (blocking) stream lags the word; querying the null stream while it
    // still counts a kernel of the library's stream as running waits for it (7-10 us, profiles/r06j),
    // so a call that follows a HIP launch first lets HIP retire it -- one stream synchronisation per
    // switch from the HIP launch to this queue, none between calls of this queue
    if (g_aql.stream_checks && w.stream_hip_busy) {
        if (hipStreamQuery(w.stream) != hipSuccess) {
            (void)hipGetLastError();
            if (hipStreamSynchronize(w.stream) != hipSuccess) return 0;
        }
        w.stream_hip_busy = false;  // until the next launch on it (coll.cpp pick_stream)
    }
    if (g_aql.stream_checks && hipStreamQuery(nullptr) != hipSuccess) {
        (void)hipGetLastError();
        ++g_aql.skip_null;
        return 0;
    }
    hsa_queue_t *q = g_aql.queue;
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
    }
    const uint64_t seq = ++w.done_seq;
    TinyArgs *a = (TinyArgs *)(g_aql.kernarg + (idx % kRing) * kSlot);
    a->in = in;
    a->io = io;
    a->count = (uint32_t)count;
    a->pad = 0;
    a->flag = w.done_flag;
    a->seq = seq;
    hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
    p->workgroup_size_x = 64;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = 64;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = ko.private_bytes;
    p->group_segment_size = ko.group_bytes;
    p->kernel_object = ko.object;
    p->kernarg_address = a;
    p->reserved2 = 0;
    p->completion_signal.handle = 0;
    const int acquire = aql_acquire_scope();
    const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                       (1 << HSA_PACKET_HEADER_BARRIER) |
                                       (acquire << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                       (g_aql.release << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    const uint16_t setup = (uint16_t)(1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS);
    __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
    const uint64_t t_bell = now_ns();
    // the word, as for a HIP launch; 10 s without it (or a queue error) turns the path off
    uint64_t t0 = 0;
    for (unsigned spins = 0;; ++spins) {
        if (__atomic_load_n(w.done_flag, __ATOMIC_ACQUIRE) >= seq) {
            ++g_prof_calls;
            g_prof_pre_ns += t_bell - t_entry;
            g_prof_wait_ns += now_ns() - t_bell;
            return 1;
        }
        if ((spins & 1023u) != 0) continue;
        if (g_aql.queue_error.load()) {
            MV2_ERR("aql: queue error %d on the MPI_Reduce_local fast path; using HIP launches from now on",
                    g_aql.queue_error.load());
            g_aql.state = -1;
            return -E_INTERN;
        }
        const uint64_t t = now_ns();
        if (!t0) t0 = t;
        if (t - t0 > 10000000000ull) {
            MV2_ERR("aql: MPI_Reduce_local kernel did not complete in 10 s; using HIP launches from now on");
            g_aql.state = -1;
            return -E_INTERN;
        }
    }
}

int aql_kernels() { return g_aql.state == 1 ? g_aql.kernels : 0; }
// the acquire scope the queue's dispatches take (HSA_FENCE_SCOPE_*: 1 agent, 2 system); -1 path off
int aql_acquire_scope() {
    if (g_aql.state != 1) return -1;
    return g_aql.acquire_set >= 0 ? g_aql.acquire_set : world().gsize > 1 ? (int)HSA_FENCE_SCOPE_SYSTEM : g_aql.acquire;
}
long aql_skips(int which) { return (long)(which ? g_aql.skip_null : g_aql.skip_lib); }

void aql_finalize() {
    if ((g_prof_calls || g_aql.skip_lib || g_aql.skip_null) && getenv("MV2AMD_HOST_PROFILE"))
        fprintf(stderr, "[mv2amd rank %d] aql profile: %llu calls, entry->doorbell %.3f us, doorbell->word %.3f us; "
                        "HIP launches instead: %llu (library words pending), %llu (null stream busy)\n",
                log_rank(), (unsigned long long)g_prof_calls, g_prof_pre_ns / 1e3 / (g_prof_calls ? g_prof_calls : 1),
                g_prof_wait_ns / 1e3 / (g_prof_calls ? g_prof_calls : 1), (unsigned long long)g_aql.skip_lib,
                (unsigned long long)g_aql.skip_null);
    const bool up = g_aql.hsa_ref;
    g_aql.hsa_ref = false;
    if (g_aql.queue) hsa_queue_destroy(g_aql.queue);
    if (g_aql.kernarg) hsa_memory_free(g_aql.kernarg);
    g_aql.queue = nullptr;
    g_aql.kernarg = nullptr;
    g_aql.state = 0;
    g_aql.kernels = 0;
    for (auto &row : g_aql.k)
        for (auto &o : row) o = KObj{};
    if (up) hsa_shut_down();  // aql_init's reference
}

}  // namespace mv2
