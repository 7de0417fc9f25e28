// launch_probe.hip — host-side cost of one blocking device call on MI355X:
// launch + hipStreamSynchronize vs launch + spin on a kernel-written pinned
// host flag, hipPointerGetAttributes, hipEventRecord.
// Build: hipcc --offload-arch=gfx950 -O2 tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_empty(int *p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] += 0;
}
__global__ void k_flag(volatile unsigned *flag, unsigned v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store((unsigned *)flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t st;
    hipStreamCreate(&st);
    int *d;
    hipMalloc(&d, 4096);
    unsigned *flag;
    hipHostMalloc((void **)&flag, 64, hipHostMallocDefault);
    *flag = 0;
    const int N = 2000;
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, d);
    hipStreamSynchronize(st);
    double t0 = now_us();
    for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, d);
        hipStreamSynchronize(st);
    }
    double a = (now_us() - t0) / N;
    t0 = now_us();
    for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, flag, (unsigned)(i + 1));
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != (unsigned)(i + 1)) {
        }
    }
    double b = (now_us() - t0) / N;
    hipStreamSynchronize(st);
    t0 = now_us();
    for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, flag, (unsigned)(N + i + 1));
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != (unsigned)(N + i + 1)) {
        }
        hipStreamSynchronize(st);
    }
    double c = (now_us() - t0) / N;
    t0 = now_us();
    hipPointerAttribute_t at;
    for (int i = 0; i < N; ++i) hipPointerGetAttributes(&at, d);
    double e = (now_us() - t0) / N;
    hipEvent_t e0;
    hipEventCreate(&e0);
    t0 = now_us();
    for (int i = 0; i < N; ++i) {
        hipEventRecord(e0, st);
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, d);
        hipStreamSynchronize(st);
    }
    double f = (now_us() - t0) / N;
    t0 = now_us();
    for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, d);
        while (hipStreamQuery(st) == hipErrorNotReady) {
        }
    }
    double g = (now_us() - t0) / N;
    printf("{\"launch_sync_us\": %.2f, \"launch_flagspin_us\": %.2f, \"flagspin_then_sync_us\": %.2f, "
           "\"ptr_attr_us\": %.3f, \"event_launch_sync_us\": %.2f, \"launch_query_spin_us\": %.2f}\n",
           a, b, c, e, f, g);
    return 0;
}
