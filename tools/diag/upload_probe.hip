// Diagnosis (not product code): after hipMemcpy host -> device from pageable memory returns, does
// a hipMemcpy device -> host of the same bytes (and a kernel reading them) see the new data?
// Several processes at once load the copy engines.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <vector>

__global__ void k_check(const unsigned *p, size_t n, unsigned seed, unsigned *bad) {
    unsigned b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != seed * 2654435761u + (unsigned)i;
    if (b) atomicAdd(bad, b);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 1000;
    const size_t n = (argc > 2 ? (size_t)atol(argv[2]) : (4u << 20)) / 4;
    unsigned *d, *bad;
    hipStream_t A;
    if (hipMalloc(&d, n * 4) || hipMalloc(&bad, 4) || hipStreamCreate(&A)) return 2;
    std::vector<unsigned> h(n), back(n);
    long wrong_d2h = 0, wrong_kernel = 0, healed = 0;
    for (int k = 1; k <= iters; ++k) {
        for (size_t i = 0; i < n; ++i) h[i] = (unsigned)k * 2654435761u + (unsigned)i;
        if (hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice)) return 3;
        // a kernel on a blocking stream right away (what a collective's first kernel does)
        if (hipMemsetAsync(bad, 0, 4, A)) return 4;
        hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, A, d, n, (unsigned)k, bad);
        unsigned hb = 0;
        if (hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, A) || hipStreamSynchronize(A)) return 5;
        if (hb) ++wrong_kernel;
        if (hipMemcpy(back.data(), d, n * 4, hipMemcpyDeviceToHost)) return 6;
        if (memcmp(back.data(), h.data(), n * 4)) {
            ++wrong_d2h;
            hipDeviceSynchronize();
            usleep(2000);
            if (hipMemcpy(back.data(), d, n * 4, hipMemcpyDeviceToHost)) return 7;
            healed += !memcmp(back.data(), h.data(), n * 4);
        }
    }
    printf("{\"iters\": %d, \"bytes\": %zu, \"wrong_kernel\": %ld, \"wrong_d2h\": %ld, \"healed_later\": %ld}\n", iters,
           n * 4, wrong_kernel, wrong_d2h, healed);
    return 0;
}
