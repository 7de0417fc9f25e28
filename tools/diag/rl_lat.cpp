// Diagnosis (not product code): where the 8-byte MPI_Reduce_local's microseconds go.
//   rl_lat lib  [iters]  -- MPI_Reduce_local SUM on 2 MPI_UNSIGNED device elements, blocking, from C
//                           (bench.py times the same call through ctypes)
//   rl_lat floor [iters] -- the platform's floor without the library: an empty one-workgroup kernel
//                           (a) + hipStreamSynchronize, (b) whose lane 0 raises a pinned host word
//                           with a system-scope release, the host spinning on the word, (c) as (b)
//                           with a relaxed word store after an explicit vmcnt wait (no L2 write-back)
// Prints one JSON line: mean and percentiles of the per-call host wall time in microseconds.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <vector>

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include "mpi.h"

static double now_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void report(const char *what, std::vector<double> &v) {
    std::sort(v.begin(), v.end());
    double s = 0;
    for (double x : v) s += x;
    printf("{\"what\": \"%s\", \"calls\": %zu, \"mean_us\": %.3f, \"p10_us\": %.3f, \"p50_us\": %.3f, \"p90_us\": %.3f}\n",
           what, v.size(), s / v.size(), v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10]);
    fflush(stdout);
}

__global__ void k_empty(unsigned *p) {
    if (threadIdx.x == 0 && p) p[1] += p[0];
}
__global__ void k_word512(unsigned *p, unsigned long long *flag, unsigned long long seq) {
    if (threadIdx.x < 2) p[2 + threadIdx.x] += p[threadIdx.x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_word(unsigned *p, unsigned long long *flag, unsigned long long seq, int light) {
    if (threadIdx.x == 0) {
        p[1] += p[0];
        if (light) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// the payload written through to memory (system-scope relaxed stores: the line leaves this XCD's L2
// with the store), then the word after the wave's stores are acknowledged: no L2 write-back
__global__ void k_word_wt(unsigned *p, unsigned long long *flag, unsigned long long seq, int) {
    if (threadIdx.x == 0) {
        __hip_atomic_store(p + 1, p[1] + p[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

void load_word_pl(unsigned *p, unsigned long long *flag, hipStream_t st);  // rl_lat_pl.hip

// ---- raw AQL dispatch of k_word from this program's own code object (mode "aql") ----
static hsa_agent_t g_agent;
static uint64_t g_kobj, g_tiny, g_wt, g_pl;
static hsa_status_t pick_gpu(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU) {
        g_agent = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t sym(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void *) {
    hsa_symbol_kind_t k;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &k);
    if (k != HSA_SYMBOL_KIND_KERNEL) return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
    char name[512] = {0};
    if (len < 500) hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, name);
    if (strstr(name, "k_wordPj")) hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &g_kobj);
    if (strstr(name, "k_word_wtPj")) hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &g_wt);
    if (strstr(name, "k_word_plPj")) hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &g_pl);
    if (strstr(name, "k_reduce_local_tinyINS_1RILi2ELi5E"))  // the library's one-wave SUM on MPI_UNSIGNED
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &g_tiny);
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t exe(hsa_executable_t e, void *) {
    hsa_executable_iterate_agent_symbols(e, g_agent, sym, nullptr);
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t karg_region(hsa_region_t r, void *d) {
    uint32_t f = 0;
    hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &f);
    if (f & HSA_REGION_GLOBAL_FLAG_KERNARG) {
        *(hsa_region_t *)d = r;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

static int aql_mode(int iters) {
    if (MPI_Init(nullptr, nullptr)) return 2;  // loads the library's code objects (its tiny kernel below)
    std::vector<double> v(iters);
    unsigned *p = nullptr;
    unsigned long long *flag = nullptr;
    hipStream_t st;
    if (hipMalloc(&p, 64) || hipMemset(p, 0, 64) || hipHostMalloc((void **)&flag, 64, hipHostMallocDefault) ||
        hipStreamCreate(&st))
        return 3;
    *flag = 0;
    hipLaunchKernelGGL(k_word, dim3(1), dim3(64), 0, st, p, flag, 1ull, 0);  // loads the code object
    load_word_pl(p, flag, st);  // and rl_lat_pl.hip's
    hipStreamSynchronize(st);
    // host cost of the ordering checks the library's fast path makes
    for (int i = 0; i < iters; ++i) {
        const double t0 = now_us();
        hipStreamQuery(st);
        v[i] = now_us() - t0;
    }
    report("hipStreamQuery(idle blocking stream)", v);
    for (int i = 0; i < iters; ++i) {
        const double t0 = now_us();
        hipStreamQuery(nullptr);
        v[i] = now_us() - t0;
    }
    report("hipStreamQuery(null stream, idle)", v);
    hsa_init();
    hsa_iterate_agents(pick_gpu, nullptr);
    hsa_ven_amd_loader_1_03_pfn_t ldr{};
    if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(ldr), &ldr) != HSA_STATUS_SUCCESS) return 4;
    ldr.hsa_ven_amd_loader_iterate_executables(exe, nullptr);
    if (!g_kobj) {
        printf("{\"error\": \"k_word kernel object not found\"}\n");
        return 5;
    }
    hsa_region_t kr{};
    hsa_agent_iterate_regions(g_agent, karg_region, &kr);
    char *karg = nullptr;
    hsa_queue_t *q = nullptr;
    if (hsa_memory_allocate(kr, 64 * 64, (void **)&karg) || hsa_queue_create(g_agent, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr,
                                                                              nullptr, UINT32_MAX, UINT32_MAX, &q))
        return 6;
    struct Args {
        unsigned *p;
        unsigned long long *flag;
        unsigned long long seq;
        int light, pad;
    };
    unsigned long long seq = 1000;
    const int scopes[4][2] = {{HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_SYSTEM},
                              {HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT},
                              {HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_NONE},
                              {HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_NONE}};
    const char *names[4] = {"AQL dispatch (acquire system, release system) + host word",
                            "AQL dispatch (acquire agent, release agent) + host word",
                            "AQL dispatch (acquire agent, release none) + host word",
                            "AQL dispatch (acquire system, release none) + host word"};
    for (int sc = 0; sc < 4; ++sc) {
        for (int i = -200; i < iters; ++i) {
            const double t0 = now_us();
            const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
            Args *a = (Args *)(karg + (idx % 64) * 64);
            a->p = p;
            a->flag = flag;
            a->seq = ++seq;
            a->light = 0;
            hsa_kernel_dispatch_packet_t *k = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
            k->workgroup_size_x = 64;
            k->workgroup_size_y = k->workgroup_size_z = 1;
            k->reserved0 = 0;
            k->grid_size_x = 64;
            k->grid_size_y = k->grid_size_z = 1;
            k->private_segment_size = 0;
            k->group_segment_size = 0;
            k->kernel_object = g_kobj;
            k->kernarg_address = a;
            k->reserved2 = 0;
            k->completion_signal.handle = 0;
            const uint16_t h = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                          (1 << HSA_PACKET_HEADER_BARRIER) |
                                          (scopes[sc][0] << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                          (scopes[sc][1] << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
            __atomic_store_n((uint32_t *)k, (uint32_t)h | (1u << 16), __ATOMIC_RELEASE);
            hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
            const double t1 = now_us();
            uint64_t spins = 0;
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < seq)
                if (++spins > 4000000000ull) {
                    printf("{\"error\": \"AQL word never arrived\"}\n");
                    return 7;
                }
            if (i >= 0) v[i] = now_us() - t0;
            (void)t1;
        }
        report(names[sc], v);
    }
    // the word kernel's variants, acquire agent / release none: (a) system-release word (as above),
    // (b) plain payload + relaxed word after vmcnt (not a valid hand-off: the floor without any L2
    // write-back), (c) write-through payload + relaxed word after vmcnt (valid), (d) (a) with
    // kernel-argument preloading
    {
        const uint64_t objs[4] = {g_kobj, g_kobj, g_wt, g_pl};
        const int light[4] = {0, 1, 0, 0};
        const char *vn[4] = {"AQL agent/none: k_word system-release word", "AQL agent/none: k_word plain payload, relaxed word (floor)",
                             "AQL agent/none: k_word_wt write-through payload, relaxed word",
                             "AQL agent/none: k_word_pl (kernarg preload) system-release word"};
        for (int rep = 0; rep < 2; ++rep)
            for (int vi = 0; vi < 4; ++vi) {
                if (!objs[vi]) {
                    printf("{\"note\": \"%s: kernel object not found\"}\n", vn[vi]);
                    continue;
                }
                for (int i = -200; i < iters; ++i) {
                    const double t0 = now_us();
                    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
                    Args *a = (Args *)(karg + (idx % 64) * 64);
                    a->p = p;
                    a->flag = flag;
                    a->seq = ++seq;
                    a->light = light[vi];
                    hsa_kernel_dispatch_packet_t *k = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
                    k->workgroup_size_x = 64;
                    k->workgroup_size_y = k->workgroup_size_z = 1;
                    k->reserved0 = 0;
                    k->grid_size_x = 64;
                    k->grid_size_y = k->grid_size_z = 1;
                    k->private_segment_size = 0;
                    k->group_segment_size = 0;
                    k->kernel_object = objs[vi];
                    k->kernarg_address = a;
                    k->reserved2 = 0;
                    k->completion_signal.handle = 0;
                    const uint16_t h = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                                  (1 << HSA_PACKET_HEADER_BARRIER) |
                                                  (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                                  (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
                    __atomic_store_n((uint32_t *)k, (uint32_t)h | (1u << 16), __ATOMIC_RELEASE);
                    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
                    uint64_t spins = 0;
                    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < seq)
                        if (++spins > 4000000000ull) {
                            printf("{\"error\": \"%s: word never arrived\"}\n", vn[vi]);
                            return 7;
                        }
                    if (i >= 0) v[i] = now_us() - t0;
                }
                report(vn[vi], v);
            }
        // the payload of the last calls: every variant computes p[1] += p[0] on zeros
        unsigned hp[4] = {9, 9, 9, 9};
        hipMemcpy(hp, p, 16, hipMemcpyDeviceToHost);
        printf("{\"payload_after\": [%u, %u]}\n", hp[0], hp[1]);
    }
    // the library's k_reduce_local_tiny (SUM, 2 x uint32) dispatched the same way, system acquire,
    // no release: the kernel object's own cost beside k_word's
    if (g_tiny) {
        unsigned *b = nullptr;
        if (hipMalloc(&b, 64) || hipMemset(b, 0, 64)) return 8;
        struct TArgs {
            const void *in;
            void *io;
            unsigned count, pad;
            unsigned long long *flag;
            unsigned long long seq;
        };
        // variant 2: kernel arguments in device memory the host writes through the BAR (what
        // HIP_FORCE_DEV_KERNARG does for HIP launches), system acquire
        char *dkarg = nullptr;
        {
            struct PoolFind {
                hsa_amd_memory_pool_t pool;
                bool found;
            } pf{{0}, false};
            hsa_amd_agent_iterate_memory_pools(
                g_agent,
                [](hsa_amd_memory_pool_t pl, void *d) -> hsa_status_t {
                    hsa_amd_segment_t seg;
                    hsa_amd_memory_pool_get_info(pl, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
                    uint32_t fl = 0;
                    hsa_amd_memory_pool_get_info(pl, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
                    if (seg == HSA_AMD_SEGMENT_GLOBAL && (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) {
                        ((PoolFind *)d)->pool = pl;
                        ((PoolFind *)d)->found = true;
                        return HSA_STATUS_INFO_BREAK;
                    }
                    return HSA_STATUS_SUCCESS;
                },
                &pf);
            hsa_agent_t cpu{};
            hsa_iterate_agents(
                [](hsa_agent_t a, void *d) -> hsa_status_t {
                    hsa_device_type_t t;
                    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
                    if (t == HSA_DEVICE_TYPE_CPU) {
                        *(hsa_agent_t *)d = a;
                        return HSA_STATUS_INFO_BREAK;
                    }
                    return HSA_STATUS_SUCCESS;
                },
                &cpu);
            if (pf.found && hsa_amd_memory_pool_allocate(pf.pool, 64 * 64, 0, (void **)&dkarg) == HSA_STATUS_SUCCESS) {
                if (hsa_amd_agents_allow_access(1, &cpu, nullptr, dkarg) != HSA_STATUS_SUCCESS) dkarg = nullptr;
            } else {
                dkarg = nullptr;
            }
            if (!dkarg) printf("{\"note\": \"no host-visible device kernarg memory\"}\n");
        }
        for (int sc = 0; sc < (dkarg ? 3 : 2); ++sc) {
            for (int i = -200; i < iters; ++i) {
                const double t0 = now_us();
                const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
                TArgs *a = (TArgs *)((sc == 2 ? dkarg : karg) + (idx % 64) * 64);
                a->in = p;
                a->io = b;
                a->count = 2;
                a->pad = 0;
                a->flag = flag;
                a->seq = ++seq;
                if (sc == 2) {  // the BAR writes land before the doorbell: fence and read one back
                    __atomic_thread_fence(__ATOMIC_SEQ_CST);
                    (void)*(volatile unsigned long long *)&a->seq;
                }
                hsa_kernel_dispatch_packet_t *k = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
                k->workgroup_size_x = 64;
                k->workgroup_size_y = k->workgroup_size_z = 1;
                k->reserved0 = 0;
                k->grid_size_x = 64;
                k->grid_size_y = k->grid_size_z = 1;
                k->private_segment_size = 0;
                k->group_segment_size = 0;
                k->kernel_object = g_tiny;
                k->kernarg_address = a;
                k->reserved2 = 0;
                k->completion_signal.handle = 0;
                const int acq = sc == 1 ? HSA_FENCE_SCOPE_AGENT : HSA_FENCE_SCOPE_SYSTEM;
                const uint16_t h = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                              (1 << HSA_PACKET_HEADER_BARRIER) | (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE));
                __atomic_store_n((uint32_t *)k, (uint32_t)h | (1u << 16), __ATOMIC_RELEASE);
                hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
                uint64_t spins = 0;
                while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < seq)
                    if (++spins > 4000000000ull) return 9;
                if (i >= 0) v[i] = now_us() - t0;
            }
            report(sc == 2 ? "AQL dispatch of libmpi k_reduce_local_tiny (system acquire, kernargs in device memory)"
                   : sc ? "AQL dispatch of libmpi k_reduce_local_tiny (agent acquire)"
                        : "AQL dispatch of libmpi k_reduce_local_tiny (system acquire)", v);
        }
    }
    hsa_queue_destroy(q);
    MPI_Finalize();
    return 0;
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "lib";
    const int iters = argc > 2 ? atoi(argv[2]) : 5000;
    if (!strcmp(mode, "aql")) return aql_mode(iters);
    std::vector<double> v(iters);
    if (!strcmp(mode, "lib")) {
        if (MPI_Init(nullptr, nullptr)) return 2;
        unsigned *a = nullptr, *b = nullptr;
        if (hipMalloc(&a, 8) || hipMalloc(&b, 8) || hipMemset(a, 0, 8) || hipMemset(b, 0, 8)) return 3;
        for (int i = 0; i < 200; ++i) MPI_Reduce_local(a, b, 2, MPI_UNSIGNED, MPI_SUM);
        for (int i = 0; i < iters; ++i) {
            const double t0 = now_us();
            if (MPI_Reduce_local(a, b, 2, MPI_UNSIGNED, MPI_SUM)) return 4;
            v[i] = now_us() - t0;
        }
        report("MPI_Reduce_local 8 B (C loop)", v);
        // host costs inside the call: the pointer classification (twice per call) and the API
        // layer up to the count test
        for (int i = 0; i < iters; ++i) {
            hipPointerAttribute_t at;
            const double t0 = now_us();
            (void)hipPointerGetAttributes(&at, a);
            v[i] = now_us() - t0;
        }
        report("hipPointerGetAttributes(device pointer)", v);
        for (int i = 0; i < iters; ++i) {
            const double t0 = now_us();
            MPI_Reduce_local(a, b, 0, MPI_UNSIGNED, MPI_SUM);
            v[i] = now_us() - t0;
        }
        report("MPI_Reduce_local count 0 (API layer)", v);
        MPI_Finalize();
        return 0;
    }
    unsigned *p = nullptr;
    unsigned long long *flag = nullptr;
    hipStream_t st;
    if (hipMalloc(&p, 64) || hipMemset(p, 0, 64) || hipHostMalloc((void **)&flag, 64, hipHostMallocDefault) ||
        hipStreamCreateWithFlags(&st, hipStreamNonBlocking))
        return 3;
    *flag = 0;
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, p);
    hipStreamSynchronize(st);
    for (int i = 0; i < iters; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, p);
        hipStreamSynchronize(st);
        v[i] = now_us() - t0;
    }
    report("empty kernel + hipStreamSynchronize", v);
    unsigned long long seq = 0;
    for (int light = 0; light < 2; ++light) {
        for (int i = 0; i < iters; ++i) {
            const double t0 = now_us();
            hipLaunchKernelGGL(k_word, dim3(1), dim3(64), 0, st, p, flag, ++seq, light);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < seq) {
            }
            v[i] = now_us() - t0;
        }
        report(light ? "kernel + relaxed host word after vmcnt wait" : "kernel + system-release host word", v);
    }
    // a 512-thread workgroup (the library's k_reduce_local shape) raising the word
    for (int i = 0; i < iters; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(k_word512, dim3(1), dim3(512), 0, st, p, flag, ++seq);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < seq) {
        }
        v[i] = now_us() - t0;
    }
    report("512-thread kernel + system-release host word", v);
    // the same 64-thread kernel on a blocking stream (the library's: ordered after null-stream work)
    hipStream_t bst;
    if (hipStreamCreate(&bst)) return 3;
    for (int i = 0; i < iters; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(k_word, dim3(1), dim3(64), 0, bst, p, flag, ++seq, 0);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < seq) {
        }
        v[i] = now_us() - t0;
    }
    report("kernel + system-release host word, blocking stream", v);
    hipStreamSynchronize(bst);
    // launch cost alone: back-to-back launches without waiting
    hipStreamSynchronize(st);
    const double t0 = now_us();
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, p);
    const double t1 = now_us();
    hipStreamSynchronize(st);
    printf("{\"what\": \"hipLaunchKernel host time, back to back\", \"calls\": %d, \"mean_us\": %.3f}\n", iters,
           (t1 - t0) / iters);
    return 0;
}
