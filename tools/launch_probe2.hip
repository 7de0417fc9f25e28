// launch_probe2.hip — host time spent inside hipLaunchKernelGGL on MI355X as a
// function of the kernel-argument size, and with libmpi.so's large code object
// loaded into the process (argv[1] = path to dlopen, optional).  Each launch is
// followed by a spin on a kernel-written pinned host word, so the queue never
// backs up: "launch" = host time of the call, "total" = launch + completion.
// Build: hipcc --offload-arch=gfx950 -O2 tools/launch_probe2.hip -o tools/launch_probe2 -ldl
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

template <int B>
struct Blob {
    unsigned char b[B];
};

template <int B>
__global__ void k_flag(Blob<B> arg, unsigned *flag, unsigned v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        __hip_atomic_store(flag, v + (arg.b[0] & 0), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int B>
static void run(hipStream_t st, unsigned *flag, unsigned &seq) {
    Blob<B> a{};
    const int N = 3000;
    for (int i = 0; i < 200; ++i) {
        hipLaunchKernelGGL(k_flag<B>, dim3(1), dim3(64), 0, st, a, flag, ++seq);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        }
    }
    double tl = 0, tt = 0;
    for (int i = 0; i < N; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(k_flag<B>, dim3(1), dim3(64), 0, st, a, flag, ++seq);
        const double t1 = now_us();
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        }
        const double t2 = now_us();
        tl += t1 - t0;
        tt += t2 - t0;
    }
    printf("{\"arg_bytes\": %d, \"launch_us\": %.3f, \"total_us\": %.3f}\n", B, tl / N, tt / N);
}

int main(int argc, char **argv) {
    if (argc > 1) {
        if (!dlopen(argv[1], RTLD_NOW | RTLD_GLOBAL)) {
            printf("dlopen failed: %s\n", dlerror());
            return 1;
        }
        printf("# loaded %s\n", argv[1]);
    }
    hipStream_t st;
    hipStreamCreate(&st);
    unsigned *flag;
    hipHostMalloc((void **)&flag, 64, hipHostMallocDefault);
    *flag = 0;
    unsigned seq = 0;
    if (argc > 1) {
        // one of libmpi.so's own kernels (k_reduce_local<SUM,F32>, one workgroup, 8 bytes) by its handle
        void *h = dlsym(RTLD_DEFAULT, "_ZN3mv214k_reduce_localINS_1RILi2ELi8EvEELi2EEEvPKDv4_jPS3_mPKNT_1TEPS8_mmNS_4DoneE");
        if (!h) {
            printf("no kernel handle\n");
            return 1;
        }
        struct Done {
            unsigned *ctr;
            unsigned long long *flag;
            unsigned long long seq;
        };
        float *buf;
        unsigned *ctr;
        unsigned long long *lflag;
        hipMalloc((void **)&buf, 64);
        hipMalloc((void **)&ctr, 73 * 4096);
        hipMemset(ctr, 0, 73 * 4096);
        hipHostMalloc((void **)&lflag, 64, hipHostMallocDefault);
        *lflag = 0;
        unsigned long long lseq = 0;
        const int N = 3000;
        double tl = 0, tt = 0;
        for (int i = 0; i < N + 200; ++i) {
            const void *in = buf, *io = buf + 4;
            size_t nvec = 0, tb = 0, te = 2;
            Done d{ctr, lflag, ++lseq};
            void *args[] = {&in, &io, &nvec, &in, &io, &tb, &te, &d};
            const double t0 = now_us();
            hipLaunchKernel(h, dim3(1), dim3(512), args, 0, st);
            const double t1 = now_us();
            while (__atomic_load_n(lflag, __ATOMIC_ACQUIRE) != lseq) {
            }
            const double t2 = now_us();
            if (i >= 200) {
                tl += t1 - t0;
                tt += t2 - t0;
            }
        }
        printf("{\"kernel\": \"libmpi k_reduce_local<SUM,F32> 1 WG\", \"launch_us\": %.3f, \"total_us\": %.3f}\n", tl / N, tt / N);
    }
    run<16>(st, flag, seq);
    run<256>(st, flag, seq);
    run<424>(st, flag, seq);
    run<704>(st, flag, seq);
    run<1536>(st, flag, seq);
    hipStreamSynchronize(st);
    return 0;
}
