// copy_probe.hip — what moves the point-to-point chunks fastest on MI355X: hipMemcpyAsync (the
// runtime's engine choice) against a plain 16-byte vector copy kernel, into ordinary and into
// uncached (hipDeviceMallocUncached, the p2p arenas') device memory.  8 MiB chunks, 50 reps.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_copy(v4u *__restrict__ d, const v4u *__restrict__ s, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) d[i] = s[i];
}

static float time_it(hipStream_t st, int reps, void (*fn)(hipStream_t, void *), void *arg) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    fn(st, arg);
    hipEventRecord(a, st);
    for (int i = 0; i < reps; ++i) fn(st, arg);
    hipEventRecord(b, st);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

struct Arg {
    void *d, *s;
    size_t bytes;
    int grid;
};
static void do_memcpy(hipStream_t st, void *p) {
    Arg *a = (Arg *)p;
    hipMemcpyAsync(a->d, a->s, a->bytes, hipMemcpyDeviceToDevice, st);
}
static void do_kernel(hipStream_t st, void *p) {
    Arg *a = (Arg *)p;
    hipLaunchKernelGGL(k_copy, dim3(a->grid), dim3(256), 0, st, (v4u *)a->d, (const v4u *)a->s, a->bytes / 16);
}

int main() {
    const size_t bytes = (size_t)8 << 20;
    void *s, *d, *u;
    hipMalloc(&s, bytes);
    hipMalloc(&d, bytes);
    hipExtMallocWithFlags(&u, bytes, hipDeviceMallocUncached);
    hipMemset(s, 1, bytes);
    hipStream_t st;
    hipStreamCreate(&st);
    for (void *dst : {d, u}) {
        Arg a{dst, s, bytes, 0};
        const float m = time_it(st, 50, do_memcpy, &a);
        printf("%-9s hipMemcpyAsync D2D        %8.2f us  %7.1f GB/s\n", dst == d ? "plain" : "uncached", m * 1e3,
               bytes / (m * 1e-3) / 1e9);
        for (int g : {64, 256, 1024, 2048}) {
            a.grid = g;
            const float k = time_it(st, 50, do_kernel, &a);
            printf("%-9s copy kernel grid %5d     %8.2f us  %7.1f GB/s\n", dst == d ? "plain" : "uncached", g, k * 1e3,
                   bytes / (k * 1e-3) / 1e9);
        }
        // and the other way round: out of uncached memory (the receiver's copy-out)
        if (dst == u) {
            Arg b{d, u, bytes, 0};
            const float m2 = time_it(st, 50, do_memcpy, &b);
            printf("from uncached hipMemcpyAsync D2D    %8.2f us  %7.1f GB/s\n", m2 * 1e3, bytes / (m2 * 1e-3) / 1e9);
            b.grid = 1024;
            const float k2 = time_it(st, 50, do_kernel, &b);
            printf("from uncached copy kernel grid 1024 %8.2f us  %7.1f GB/s\n", k2 * 1e3, bytes / (k2 * 1e-3) / 1e9);
        }
    }
    return 0;
}
