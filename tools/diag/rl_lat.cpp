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

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "lib";
    const int iters = argc > 2 ? atoi(argv[2]) : 5000;
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
