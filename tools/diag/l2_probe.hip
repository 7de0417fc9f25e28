// Diagnosis (not product code): is data written by a copy on one stream, after the host has
// synchronised that stream, always seen by a kernel launched next on ANOTHER stream, when that
// kernel's XCDs read the same buffer before the copy (L2-resident old lines)?
//   mode 0: hipMemcpyAsync D2D on stream B + hipStreamSynchronize(B), check kernel on stream A
//   mode 1: the same with the check kernel on stream B (control: same stream)
//   mode 2: a copy kernel on stream B + hipStreamSynchronize(B), check kernel on stream A
//   mode 3: mode 0 with an event: hipEventRecord(ev, B); hipStreamWaitEvent(A, ev) before the check
//   host -> device (copy engine) instead of device -> device, the old lines written by a kernel on A:
//   mode 4: hipMemcpy H2D from pinned memory (null stream, synchronous), check kernel on A
//   mode 5: hipMemcpyAsync H2D from pinned memory on A itself, check kernel on A
//   mode 6: hipMemcpyAsync H2D from pinned memory on B + hipStreamSynchronize(B), check kernel on A
//   mode 7: hipMemcpy H2D from pageable memory, check kernel on A
//   mode 8: mode 4 with the old lines only read (k_touch) on A
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_fill(unsigned *p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = seed * 2654435761u + (unsigned)i;
}
__global__ void k_touch(const unsigned *p, size_t n, unsigned *sink) {  // pull every line into the L2s
    unsigned s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    if (s == 0x12345678u) sink[0] = s;
}
__global__ void k_copy(unsigned *d, const unsigned *s, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}
__global__ void k_check(const unsigned *p, size_t n, unsigned seed, unsigned *bad) {
    unsigned b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != seed * 2654435761u + (unsigned)i;
    if (b) atomicAdd(bad, b);
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0, iters = argc > 2 ? atoi(argv[2]) : 300;
    const size_t n = (3u << 20) / 4;  // 3 MiB
    unsigned *g, *src[2], *bad, *sink;
    hipStream_t A, B;
    hipEvent_t ev;
    if (hipMalloc(&g, n * 4) || hipMalloc(&src[0], n * 4) || hipMalloc(&src[1], n * 4) || hipMalloc(&bad, 4) ||
        hipMalloc(&sink, 4) || hipStreamCreate(&A) || hipStreamCreate(&B) || hipEventCreateWithFlags(&ev, hipEventDisableTiming))
        return 2;
    unsigned *hp = nullptr, *hpage = (unsigned *)malloc(n * 4);
    if (hipHostMalloc((void **)&hp, n * 4, hipHostMallocDefault)) return 2;
    long wrong_iters = 0, wrong_words = 0;
    for (int k = 0; k < iters; ++k) {
        const unsigned seed = (unsigned)k + 1;
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, B, src[k & 1], n, seed);
        if (hipStreamSynchronize(B)) return 3;
        if (mode >= 4) {
            for (size_t i = 0; i < n; ++i) hp[i] = hpage[i] = seed * 2654435761u + (unsigned)i;
            if (mode == 8) hipLaunchKernelGGL(k_touch, dim3(2048), dim3(256), 0, A, g, n, sink);
            else hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, A, g, n, seed + 7777u);  // old lines, written
            if (hipStreamSynchronize(A)) return 3;
            if (mode == 4 || mode == 8) { if (hipMemcpy(g, hp, n * 4, hipMemcpyHostToDevice)) return 4; }
            else if (mode == 5) { if (hipMemcpyAsync(g, hp, n * 4, hipMemcpyHostToDevice, A)) return 4; }
            else if (mode == 6) { if (hipMemcpyAsync(g, hp, n * 4, hipMemcpyHostToDevice, B) || hipStreamSynchronize(B)) return 4; }
            else { if (hipMemcpy(g, hpage, n * 4, hipMemcpyHostToDevice)) return 4; }
            if (hipMemsetAsync(bad, 0, 4, A)) return 6;
            hipLaunchKernelGGL(k_check, dim3(2048), dim3(256), 0, A, g, n, seed, bad);
            unsigned hb = 0;
            if (hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost)) return 7;
            if (hb) { ++wrong_iters; wrong_words += hb; }
            continue;
        }
        hipLaunchKernelGGL(k_touch, dim3(2048), dim3(256), 0, A, g, n, sink);  // old data into the L2s
        if (hipStreamSynchronize(A)) return 3;
        if (mode == 2) hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, B, g, src[k & 1], n);
        else if (hipMemcpyAsync(g, src[k & 1], n * 4, hipMemcpyDeviceToDevice, B)) return 4;
        if (mode == 3) {
            hipEventRecord(ev, B);
            hipStreamWaitEvent(A, ev, 0);
        } else if (hipStreamSynchronize(B)) return 5;
        hipStream_t cs = mode == 1 ? B : A;
        if (hipMemsetAsync(bad, 0, 4, cs)) return 6;
        hipLaunchKernelGGL(k_check, dim3(2048), dim3(256), 0, cs, g, n, seed, bad);
        unsigned hb = 0;
        if (hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost)) return 7;
        if (hb) {
            ++wrong_iters;
            wrong_words += hb;
        }
    }
    printf("{\"mode\": %d, \"iters\": %d, \"wrong_iters\": %ld, \"wrong_words\": %ld}\n", mode, iters, wrong_iters, wrong_words);
    return 0;
}
