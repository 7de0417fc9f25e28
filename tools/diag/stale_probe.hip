// Diagnosis (not product code): which acquire scope must a kernel dispatched by hand into an HSA
// queue (runtime/aql.cpp) carry so that it never reads an operand's old bytes from an L2?
// Each iteration: (1) a kernel of 8 workgroups dispatched into the probe's own queue reads all of X
// (every XCD's L2 now holds X's lines); (2) X is rewritten -- mode 0 by hipMemcpy host -> device (copy
// engine), mode 1 by a kernel on a HIP stream, followed by hipStreamSynchronize; (3) a kernel of 8
// workgroups dispatched into the probe's queue with acquire scope S checks every word of X against
// the new pattern.  S = none must be able to show stale words for the probe to mean anything; the
// question is whether S = agent ever does.
// usage: stale_probe <iters>; prints one JSON line per (mode, scope).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

constexpr size_t kWords = 16384;  // 64 KiB
constexpr int kBlocks = 8;

__global__ void k_touch(const unsigned *x, unsigned *sink) {
    unsigned s = 0;
    for (size_t i = threadIdx.x; i < kWords; i += 256) s += x[i];  // 256-thread workgroups: no hidden arguments
    if (s == 0xdeadbeefu) sink[blockIdx.x] = s;  // keeps the loads
}
__global__ void k_check(const unsigned *x, unsigned tag, unsigned long long *bad) {
    unsigned b = 0;
    for (size_t i = threadIdx.x; i < kWords; i += 256) b += x[i] != tag * 2654435761u + (unsigned)i;
    if (b) __hip_atomic_fetch_add(bad, (unsigned long long)b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_fill(unsigned *x, unsigned tag) {
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < kWords; i += gridDim.x * blockDim.x)
        x[i] = tag * 2654435761u + (unsigned)i;
}

static hsa_agent_t g_agent;
static uint64_t g_touch, g_check;
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
    if (strstr(name, "k_touch")) hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &g_touch);
    if (strstr(name, "k_check")) hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &g_check);
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

static hsa_queue_t *q;
static char *karg;
static hsa_signal_t sig;

// dispatch kernel `obj` with `args` (bytes) on kBlocks x 256, acquire scope `acq`, release system; wait
static bool dispatch(uint64_t obj, const void *args, size_t bytes, int acq) {
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    char *a = karg + (idx % 64) * 256;
    memcpy(a, args, bytes);
    hsa_signal_store_relaxed(sig, 1);
    hsa_kernel_dispatch_packet_t *k = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
    k->workgroup_size_x = 256;
    k->workgroup_size_y = k->workgroup_size_z = 1;
    k->reserved0 = 0;
    k->grid_size_x = 256 * kBlocks;
    k->grid_size_y = k->grid_size_z = 1;
    k->private_segment_size = 0;
    k->group_segment_size = 0;
    k->kernel_object = obj;
    k->kernarg_address = a;
    k->reserved2 = 0;
    k->completion_signal = sig;
    const uint16_t h = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                                  (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                  (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    __atomic_store_n((uint32_t *)k, (uint32_t)h | (1u << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
    return hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 10000000000ull, HSA_WAIT_STATE_ACTIVE) == 0;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    unsigned *x = nullptr, *sink = nullptr;
    unsigned long long *bad = nullptr;
    hipStream_t st;
    if (hipMalloc(&x, kWords * 4) || hipMalloc(&sink, 64 * 4) || hipHostMalloc((void **)&bad, 64, hipHostMallocDefault) ||
        hipStreamCreate(&st))
        return 2;
    hipLaunchKernelGGL(k_fill, dim3(8), dim3(256), 0, st, x, 0u);  // loads the code object
    hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, st, x, sink);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, st, x, 0u, bad);
    hipStreamSynchronize(st);
    hsa_init();
    hsa_iterate_agents(pick_gpu, nullptr);
    hsa_ven_amd_loader_1_03_pfn_t ldr{};
    if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(ldr), &ldr) != HSA_STATUS_SUCCESS) return 3;
    ldr.hsa_ven_amd_loader_iterate_executables(exe, nullptr);
    if (!g_touch || !g_check) {
        printf("{\"error\": \"kernel objects not found\"}\n");
        return 4;
    }
    hsa_region_t kr{};
    hsa_agent_iterate_regions(g_agent, karg_region, &kr);
    if (hsa_memory_allocate(kr, 64 * 256, (void **)&karg) || hsa_signal_create(1, 0, nullptr, &sig) ||
        hsa_queue_create(g_agent, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q))
        return 5;
    std::vector<unsigned> h(kWords);
    const int scopes[3] = {HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_SYSTEM};
    const char *sname[3] = {"none", "agent", "system"};
    unsigned tag = 1;
    for (int mode = 0; mode < 2; ++mode)
        for (int sc = 0; sc < 3; ++sc) {
            *bad = 0;
            long bad_iters = 0;
            unsigned long long last = 0;
            for (int it = 0; it < iters; ++it) {
                struct {
                    const unsigned *x;
                    unsigned *sink;
                } ta{x, sink};
                if (!dispatch(g_touch, &ta, sizeof(ta), scopes[sc])) return 6;
                ++tag;
                if (mode == 0) {
                    for (size_t i = 0; i < kWords; ++i) h[i] = tag * 2654435761u + (unsigned)i;
                    if (hipMemcpy(x, h.data(), kWords * 4, hipMemcpyHostToDevice)) return 7;
                } else {
                    hipLaunchKernelGGL(k_fill, dim3(8), dim3(256), 0, st, x, tag);
                    if (hipStreamSynchronize(st)) return 7;
                }
                struct {
                    const unsigned *x;
                    unsigned tag, pad;
                    unsigned long long *bad;
                } ca{x, tag, 0, bad};
                if (!dispatch(g_check, &ca, sizeof(ca), scopes[sc])) return 8;
                const unsigned long long b = __atomic_load_n(bad, __ATOMIC_ACQUIRE);
                if (b != last) ++bad_iters;
                last = b;
            }
            printf("{\"rewrite\": \"%s\", \"acquire\": \"%s\", \"iters\": %d, \"stale_words\": %llu, \"stale_iters\": %ld}\n",
                   mode ? "kernel on a HIP stream" : "hipMemcpy host->device", sname[sc], iters,
                   (unsigned long long)*bad, bad_iters);
            fflush(stdout);
        }
    hsa_queue_destroy(q);
    return 0;
}
