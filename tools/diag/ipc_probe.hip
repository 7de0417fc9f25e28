// Diagnosis (not product code): is data that one process's kernel stores into another process's
// uncached, IPC-imported buffer visible to the owner's kernels once the writer has published?
// Two processes (role "r" owns the buffer, role "w" writes it) share a /dev/shm control page.
// Each round the writer fills its source with pattern k, copies it into the owner's buffer with a
// kernel, completes the copy in one of three ways, then publishes k; the owner checks every word.
//   mode 0: the copy kernel's last workgroup fences (agent acq_rel + vmcnt(0)) per XCD group and
//           raises a pinned host word with a system-scope release; the host spins on the word
//   mode 1: hipStreamSynchronize after the copy kernel (no word)
//   mode 2: every workgroup fences at system scope before the word (like mode 0 otherwise)
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>
#include <atomic>

struct Ctl {
    std::atomic<long> ready, seq, ack;
    hipIpcMemHandle_t h;
};

__global__ void k_fill(unsigned *p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = seed * 2654435761u + (unsigned)i;
}
__global__ void k_copy_word(unsigned *d, const unsigned *s, size_t n, unsigned *ctr, unsigned long long *flag,
                            unsigned long long seq, int mode) {
    const size_t per = (n + gridDim.x - 1) / gridDim.x, b0 = blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    for (size_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) d[i] = s[i];  // block-contiguous, like pack
    if (mode == 1) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x) return;
    if (mode == 2) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");  // system scope, every block
    const unsigned g = blockIdx.x & 7u, members = (gridDim.x - g + 7u) / 8u, groups = gridDim.x < 8u ? gridDim.x : 8u;
    if (__hip_atomic_fetch_add(ctr + g * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u != members) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(ctr + 8 * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u != groups) return;
    for (int k = 0; k < 9; ++k) __hip_atomic_store(ctr + k * 64, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_check(const unsigned *p, size_t n, unsigned seed, unsigned *bad) {
    unsigned b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != seed * 2654435761u + (unsigned)i;
    if (b) atomicAdd(bad, b);
}

int main(int argc, char **argv) {
    if (argc < 5) return 2;
    const char role = argv[1][0];
    const int mode = atoi(argv[2]), iters = atoi(argv[3]);
    const char *shm = argv[4];
    const size_t n = (4u << 20) / 4;
    int fd = shm_open(shm, O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, sizeof(Ctl))) return 3;
    Ctl *c = (Ctl *)mmap(nullptr, sizeof(Ctl), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (role == 'r') {
        unsigned *buf, *bad;
        if (hipExtMallocWithFlags((void **)&buf, n * 4, hipDeviceMallocUncached) || hipMalloc(&bad, 4)) return 4;
        if (hipIpcGetMemHandle(&c->h, buf)) return 5;
        c->ready.store(1);
        long wrong_iters = 0, wrong_words = 0;
        for (long k = 1; k <= iters; ++k) {
            while (c->seq.load(std::memory_order_acquire) < k) {}
            hipMemset(bad, 0, 4);
            hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, 0, buf, n, (unsigned)k, bad);
            unsigned hb = 0;
            hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
            if (hb) { ++wrong_iters; wrong_words += hb; }
            c->ack.store(k, std::memory_order_release);
        }
        printf("{\"mode\": %d, \"iters\": %d, \"wrong_iters\": %ld, \"wrong_words\": %ld}\n", mode, iters, wrong_iters, wrong_words);
        shm_unlink(shm);
        return 0;
    }
    while (c->ready.load() == 0) usleep(1000);
    unsigned *dst, *src, *ctr;
    unsigned long long *flag;
    hipStream_t st;
    if (hipIpcOpenMemHandle((void **)&dst, c->h, hipIpcMemLazyEnablePeerAccess) || hipMalloc(&src, n * 4) ||
        hipMalloc(&ctr, 9 * 64 * 4) || hipMemset(ctr, 0, 9 * 64 * 4) || hipHostMalloc((void **)&flag, 8, 0) ||
        hipStreamCreate(&st))
        return 6;
    *flag = 0;
    hipDeviceSynchronize();
    for (long k = 1; k <= iters; ++k) {
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, st, src, n, (unsigned)k);
        hipLaunchKernelGGL(k_copy_word, dim3(1024), dim3(256), 0, st, dst, src, n, ctr, flag, (unsigned long long)k, mode);
        if (mode == 1) hipStreamSynchronize(st);
        else while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < (unsigned long long)k) {}
        c->seq.store(k, std::memory_order_release);
        while (c->ack.load(std::memory_order_acquire) < k) {}
    }
    hipStreamSynchronize(st);
    return 0;
}
