// Diagnosis (not product code): rl_lat's k_word compiled with kernel-argument preloading
// (-mllvm -amdgpu-kernarg-preload-count=8: the packet processor loads the first kernel-argument
// dwords into SGPRs, the wave issues no s_load for them).  Built as its own translation unit so the
// option applies to this kernel only.
#include <hip/hip_runtime.h>

__global__ void k_word_pl(unsigned *p, unsigned long long *flag, unsigned long long seq, int) {
    if (threadIdx.x == 0) {
        p[1] += p[0];
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// a HIP launch that loads this translation unit's code object (the AQL loop then finds the kernel)
void load_word_pl(unsigned *p, unsigned long long *flag, hipStream_t st) {
    hipLaunchKernelGGL(k_word_pl, dim3(1), dim3(64), 0, st, p, flag, 1ull, 0);
}
