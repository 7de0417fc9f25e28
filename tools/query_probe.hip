// query_probe.hip — host cost of asking HIP whether a stream is idle (hipStreamQuery on the
// legacy null stream / a blocking stream / a non-blocking stream, hipEventQuery) and of an
// empty-kernel launch, on an idle GPU.  Build: hipcc --offload-arch=gfx950 -O2 tools/query_probe.hip -o tools/query_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty() {}

template <class F>
static double us_per(F f, int iters) {
    for (int i = 0; i < 100; ++i) f();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) f();
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
}

int main() {
    hipStream_t sb, snb;
    hipStreamCreate(&sb);
    hipStreamCreateWithFlags(&snb, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, sb);
    hipDeviceSynchronize();
    const int N = 20000;
    printf("hipStreamQuery(null)        %.3f us\n", us_per([] { (void)hipStreamQuery(nullptr); }, N));
    printf("hipStreamQuery(blocking)    %.3f us\n", us_per([&] { (void)hipStreamQuery(sb); }, N));
    printf("hipStreamQuery(nonblocking) %.3f us\n", us_per([&] { (void)hipStreamQuery(snb); }, N));
    hipEventRecord(ev, nullptr);
    hipDeviceSynchronize();
    printf("hipEventQuery(done)         %.3f us\n", us_per([&] { (void)hipEventQuery(ev); }, N));
    printf("hipEventRecord(null)        %.3f us\n", us_per([&] { (void)hipEventRecord(ev, nullptr); }, N));
    hipDeviceSynchronize();
    printf("launch empty (blocking st)  %.3f us\n", us_per([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, sb); }, N));
    hipDeviceSynchronize();
    printf("launch+sync empty           %.3f us\n", us_per([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, sb); hipStreamSynchronize(sb); }, 2000));
    return 0;
}
