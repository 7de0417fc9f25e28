// uc_bw.hip — copy bandwidth between coarse-grained (hipMalloc) and uncached
// (hipDeviceMallocUncached, the pipeline arenas' memory type) buffers on one
// MI355X.  Decides whether arena-side loads/stores pay an uncached penalty.
//   hipcc --offload-arch=gfx950 -O3 tools/uc_bw.hip -o tools/uc_bw && tools/uc_bw
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int NT>
__global__ __launch_bounds__(256) void k_copy(const v4u *__restrict__ s, v4u *__restrict__ d, size_t nv) {
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    for (size_t i = (size_t)blockIdx.x * 256 * 4 + threadIdx.x; i < nv; i += stride) {
        v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < nv) v[u] = NT ? __builtin_nontemporal_load(s + i + u * 256) : s[i + u * 256];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < nv) {
                if (NT) __builtin_nontemporal_store(v[u], d + i + u * 256);
                else d[i + u * 256] = v[u];
            }
    }
}

int main() {
    const size_t bytes = (size_t)256 << 20, nv = bytes / 16;
    void *a, *b, *u1, *u2;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipExtMallocWithFlags(&u1, bytes, hipDeviceMallocUncached);
    hipExtMallocWithFlags(&u2, bytes, hipDeviceMallocUncached);
    hipMemset(a, 1, bytes);
    hipMemset(u1, 1, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct { const char *name; void *s, *d; } cases[] = {
        {"coarse->coarse", a, b}, {"uncached->coarse", u1, b}, {"coarse->uncached", a, u1}, {"uncached->uncached", u1, u2}};
    for (int grid : {256, 1024, 4096}) {
        for (auto &c : cases) {
            for (int nt = 0; nt < 2; ++nt) {
                auto k = nt ? k_copy<1> : k_copy<0>;
                for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, (const v4u *)c.s, (v4u *)c.d, nv);
                hipEventRecord(e0);
                const int reps = 20;
                for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, (const v4u *)c.s, (v4u *)c.d, nv);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                printf("grid %5d %-20s nt=%d  %8.1f GB/s (2 x 256 MiB per copy)\n", grid, c.name, nt,
                       2.0 * bytes * reps / (ms * 1e-3) / 1e9);
            }
        }
    }
    return 0;
}
