// Diagnosis (not product code): does workgroup b always run on the XCD of b % 8?  block_done
// (device_util.h) writes back one XCD's L2 per group of blocks with equal b % 8.  Each launch
// records every block's XCC_ID; the host counts launches where two blocks of one b % 8 group ran
// on different XCDs.  Run several processes at once to load the GPU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

__global__ void k_xcc(unsigned *out, int spin) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    if (threadIdx.x == 0) out[blockIdx.x] = x;
    // a little work so that blocks overlap other processes' kernels
    volatile float a = 1.f;
    for (int i = 0; i < spin; ++i) a = a * 1.0001f;
}

int main(int argc, char **argv) {
    const int launches = argc > 1 ? atoi(argv[1]) : 2000;
    const int grids[] = {9, 64, 256, 1000, 4096};
    unsigned *d;
    hipMalloc(&d, 4096 * sizeof(unsigned));
    std::vector<unsigned> h(4096);
    long bad = 0, total = 0, seen_off = 0;
    int first_xcc_hist[8] = {0};
    for (int k = 0; k < launches; ++k) {
        const int g = grids[k % 5];
        hipLaunchKernelGGL(k_xcc, dim3(g), dim3(256), 0, 0, d, (k % 3) * 200);
        hipMemcpy(h.data(), d, g * sizeof(unsigned), hipMemcpyDeviceToHost);
        bool ok = true;
        for (int b = 8; b < g; ++b)
            if (h[b] != h[b % 8]) ok = false;
        first_xcc_hist[h[0] & 7]++;
        if (h[0] != 0) ++seen_off;
        bad += !ok;
        ++total;
    }
    printf("{\"launches\": %ld, \"groups_split\": %ld, \"block0_not_xcc0\": %ld, \"block0_xcc_hist\": [%d,%d,%d,%d,%d,%d,%d,%d]}\n",
           total, bad, seen_off, first_xcc_hist[0], first_xcc_hist[1], first_xcc_hist[2], first_xcc_hist[3],
           first_xcc_hist[4], first_xcc_hist[5], first_xcc_hist[6], first_xcc_hist[7]);
    return 0;
}
