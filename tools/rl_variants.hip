// rl_variants.hip — micro-benchmark of Reduce_local (fp32 SUM, 256 MiB)
// kernel shapes on one MI355X, to pick the product kernel's configuration.
// Build: hipcc --offload-arch=gfx950 -O3 tools/rl_variants.hip -o tools/rl_variants
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>
#include <random>

#include "../mvapich2_amd/csrc/device_util.h"

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int U, bool LNT, bool SNT, int T>
__global__ __launch_bounds__(T) void k_rl(const v4f *__restrict__ in, v4f *__restrict__ io, size_t nvec) {
    const size_t stride = (size_t)gridDim.x * T * U;
    for (size_t base = (size_t)blockIdx.x * T * U + threadIdx.x; base < nvec; base += stride) {
        v4f a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < nvec) {
                if (LNT) {
                    a[u] = __builtin_nontemporal_load(&io[i]);
                    b[u] = __builtin_nontemporal_load(&in[i]);
                } else {
                    a[u] = io[i];
                    b[u] = in[i];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < nvec) {
                v4f r = a[u] + b[u];
                if (SNT) __builtin_nontemporal_store(r, &io[i]);
                else io[i] = r;
            }
        }
    }
}

// product shape + the completion-word epilogue (device_util.h block_done)
template <int U, int T>
__global__ __launch_bounds__(T) void k_rl_done(const v4f *__restrict__ in, v4f *__restrict__ io, size_t nvec,
                                               mv2::Done dn) {
    const size_t stride = (size_t)gridDim.x * T * U;
    for (size_t base = (size_t)blockIdx.x * T * U + threadIdx.x; base < nvec; base += stride) {
        v4f a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < nvec) {
                a[u] = __builtin_nontemporal_load(&io[i]);
                b[u] = __builtin_nontemporal_load(&in[i]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < nvec) __builtin_nontemporal_store(a[u] + b[u], &io[i]);
        }
    }
    mv2::block_done(dn);
}

// contiguous chunk per workgroup (better DRAM page locality than grid-stride)
template <int U, int T>
__global__ __launch_bounds__(T) void k_rl_chunk(const v4f *__restrict__ in, v4f *__restrict__ io, size_t nvec,
                                                size_t chunk) {
    const size_t beg = (size_t)blockIdx.x * chunk;
    const size_t end = beg + chunk < nvec ? beg + chunk : nvec;
    for (size_t base = beg + threadIdx.x; base < end; base += (size_t)T * U) {
        v4f a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < end) {
                a[u] = __builtin_nontemporal_load(&io[i]);
                b[u] = __builtin_nontemporal_load(&in[i]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < end) __builtin_nontemporal_store(a[u] + b[u], &io[i]);
        }
    }
}

// read-only ceiling: 2 read streams, one tiny write per thread
template <int U, int T>
__global__ __launch_bounds__(T) void k_read2(const v4f *__restrict__ in, const v4f *__restrict__ io, size_t nvec,
                                             v4f *sink) {
    v4f acc = {0, 0, 0, 0};
    const size_t stride = (size_t)gridDim.x * T * U;
    for (size_t base = (size_t)blockIdx.x * T * U + threadIdx.x; base < nvec; base += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < nvec) acc += __builtin_nontemporal_load(&io[i]) + __builtin_nontemporal_load(&in[i]);
        }
    }
    if (acc.x == 12345.f) sink[threadIdx.x] = acc;
}

// pure copy (1 read + 1 write stream): the bandwidth ceiling reference
template <int U, int T>
__global__ __launch_bounds__(T) void k_copy(const v4f *__restrict__ in, v4f *__restrict__ out, size_t nvec) {
    const size_t stride = (size_t)gridDim.x * T * U;
    for (size_t base = (size_t)blockIdx.x * T * U + threadIdx.x; base < nvec; base += stride) {
        v4f a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < nvec) a[u] = in[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            if (i < nvec) __builtin_nontemporal_store(a[u], &out[i]);
        }
    }
}

template <class F>
static float timeit(F f, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> v;
    for (int i = 0; i < 3; ++i) f();
    for (int i = 0; i < iters; ++i) {
        hipEventRecord(e0);
        f();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const size_t S = 256ull << 20, nvec = S / 16;
    v4f *a, *b, *c;
    hipMalloc(&a, S);
    hipMalloc(&b, S);
    hipMalloc(&c, S);
    {
        // random operands (zero-filled buffers measured faster than HBM peak: not representative)
        std::vector<float> h(S / 4);
        std::mt19937 g(5);
        std::uniform_real_distribution<float> U(-1.f, 1.f);
        for (auto &x : h) x = U(g);
        hipMemcpy(a, h.data(), S, hipMemcpyHostToDevice);
        for (auto &x : h) x = U(g);
        hipMemcpy(b, h.data(), S, hipMemcpyHostToDevice);
        hipMemcpy(c, h.data(), S, hipMemcpyHostToDevice);
    }
    auto report = [&](const char *name, int grid, float ms, double bytes) {
        printf("%-34s grid=%7d  %.4f ms  %7.1f GB/s\n", name, grid, ms, bytes / ms / 1e6);
    };
#define RUN(NAME, U, LNT, SNT, T, GRID)                                                                   \
    {                                                                                                     \
        int g = GRID;                                                                                     \
        if (g <= 0) g = (int)((nvec + (size_t)T * U - 1) / ((size_t)T * U));                             \
        float ms = timeit([&] { hipLaunchKernelGGL((k_rl<U, LNT, SNT, T>), dim3(g), dim3(T), 0, 0, a, b, nvec); }, 20); \
        report(NAME, g, ms, 3.0 * S);                                                                     \
    }
    for (int grid : {4096, 8192, 0}) {
        RUN("U4 ld_nt st_nt   256", 4, true, true, 256, grid);
        RUN("U4 ld_nt st      256", 4, true, false, 256, grid);
        RUN("U4 ld    st      256", 4, false, false, 256, grid);
        RUN("U2 ld_nt st_nt   512", 2, true, true, 512, grid);
        RUN("U2 ld_nt st      512", 2, true, false, 512, grid);
    }
    {
        uint32_t *ctr;
        hipMalloc(&ctr, mv2::kDoneBytes);
        hipMemset(ctr, 0, mv2::kDoneBytes);
        uint64_t *flag;
        hipHostMalloc((void **)&flag, 64, hipHostMallocDefault);
        uint64_t seq = 0;
        for (int grid : {4096, 8192, 16384}) {
            float ms = timeit([&] {
                mv2::Done dn{ctr, flag, ++seq};
                hipLaunchKernelGGL((k_rl_done<4, 256>), dim3(grid), dim3(256), 0, 0, a, b, nvec, dn);
            }, 20);
            report("U4 nt/nt 256 + block_done", grid, ms, 3.0 * S);
        }
    }
    for (int grid : {1024, 4096}) {
        float ms = timeit([&] { hipLaunchKernelGGL((k_read2<4, 256>), dim3(grid), dim3(256), 0, 0, a, b, nvec, c); }, 20);
        report("read2 U4 nt (2R ceiling)", grid, ms, 2.0 * S);
    }
    for (int grid : {2048, 0}) {
        int g = grid ? grid : (int)(nvec / 1024);
        float ms = timeit([&] { hipLaunchKernelGGL((k_copy<4, 256>), dim3(g), dim3(256), 0, 0, a, c, nvec); }, 20);
        report("copy U4 (1R+1W ceiling)", g, ms, 2.0 * S);
    }
    return 0;
}
