// pack_variants.hip — micro-benchmark of MPI_Pack / MPI_Unpack kernel shapes on the
// configs[4] layout MPI_Type_vector(8Mi, 4, 8, MPI_FLOAT) (16-byte blocks every 32 bytes,
// 128 MiB packed, 256 MiB span) on one MI355X, to pick the product kernel's shape.
// Build: hipcc --offload-arch=gfx950 -O3 tools/pack_variants.hip -o tools/pack_variants
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../mvapich2_amd/csrc/device_util.h"  // mv2::Done / block_done: the product's completion word

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

// strided units: row i at src + i*su (in 16-byte units), one 16-byte unit per row
template <int U, int T, bool LNT, bool SNT, bool UNPACK>
__global__ __launch_bounds__(T) void k_units(const v4u *__restrict__ src, v4u *__restrict__ dst, size_t rows,
                                             size_t su) {
    const size_t base = (size_t)blockIdx.x * T * U + threadIdx.x;
    v4u v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const size_t u = base + (size_t)k * T;
        if (u < rows) {
            const v4u *p = src + (UNPACK ? u : u * su);
            v[k] = LNT ? __builtin_nontemporal_load(p) : *p;
        }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const size_t u = base + (size_t)k * T;
        if (u < rows) {
            v4u *q = dst + (UNPACK ? u * su : u);
            if (SNT) __builtin_nontemporal_store(v[k], q);
            else *q = v[k];
        }
    }
}

// grid-stride version (fixed grid, U units in flight per thread per iteration)
template <int U, int T, bool SNT, bool UNPACK>
__global__ __launch_bounds__(T) void k_units_gs(const v4u *__restrict__ src, v4u *__restrict__ dst, size_t rows,
                                                size_t su) {
    const size_t step = (size_t)gridDim.x * T * U;
    for (size_t base = (size_t)blockIdx.x * T * U + threadIdx.x; base < rows; base += step) {
        v4u v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const size_t u = base + (size_t)k * T;
            if (u < rows) v[k] = __builtin_nontemporal_load(src + (UNPACK ? u : u * su));
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const size_t u = base + (size_t)k * T;
            if (u < rows) {
                v4u *q = dst + (UNPACK ? u * su : u);
                if (SNT) __builtin_nontemporal_store(v[k], q);
                else *q = v[k];
            }
        }
    }
}

// pack with contiguous span loads (stride = 2 units): each lane loads 16 bytes of the span
// contiguously (full lines, no half-used lines per instruction), then the payload lanes are
// compacted across the wave with ds_bpermute: output lane j takes span lane 2j (first load)
// or 2j-64 (second load).
template <int T, bool SNT>
__global__ __launch_bounds__(T) void k_pack_perm2(const v4u *__restrict__ src, v4u *__restrict__ dst, size_t rows) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * T + threadIdx.x) >> 6;  // 64 rows per wave
    const size_t r0 = wave * 64;
    if (r0 >= rows) return;
    const v4u *s = src + r0 * 2;  // span of 64 rows = 128 units
    const size_t lim = (rows - r0) * 2;
    v4u a = (size_t)lane < lim ? __builtin_nontemporal_load(s + lane) : v4u{0, 0, 0, 0};
    v4u b = (size_t)(lane + 64) < lim ? __builtin_nontemporal_load(s + 64 + lane) : v4u{0, 0, 0, 0};
    const int srcl = (2 * lane) & 63;
    const bool hi = lane >= 32;
    v4u r;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int xa = __builtin_amdgcn_ds_bpermute(srcl * 4, (int)a[c]);
        const int xb = __builtin_amdgcn_ds_bpermute(srcl * 4, (int)b[c]);
        r[c] = (unsigned)(hi ? xb : xa);
    }
    if (r0 + lane < rows) {
        if (SNT) __builtin_nontemporal_store(r, dst + r0 + lane);
        else dst[r0 + lane] = r;
    }
}

// write-only references over the 256 MiB span: every 16-byte unit (whole lines), or the first
// 16 bytes of every 32-byte sector (the unpack's byte-masked write pattern without its reads)
template <int T, bool HALF>
__global__ __launch_bounds__(T) void k_write_only(v4u *__restrict__ dst, size_t units) {
    const size_t u = (size_t)blockIdx.x * T + threadIdx.x;
    if (u < units) dst[HALF ? 2 * u : u] = v4u{(unsigned)u, 1u, 2u, 3u};
}
// read the packed 128 MiB and write whole 32-byte sectors (payload + zeroed gap): the traffic an
// unpack would have if it were allowed to overwrite the gaps (not a valid MPI_Unpack)
template <int T>
__global__ __launch_bounds__(T) void k_expand_whole(const v4u *__restrict__ src, v4u *__restrict__ dst, size_t rows) {
    const size_t u = (size_t)blockIdx.x * T + threadIdx.x;
    if (u < rows) {
        const v4u v = __builtin_nontemporal_load(src + u);
        dst[2 * u] = v;
        dst[2 * u + 1] = v4u{0xA5A5A5A5u, 0xA5A5A5A5u, 0xA5A5A5A5u, 0xA5A5A5A5u};
    }
}
// unpack, one row per lane but each workgroup owning a contiguous 1/8th-of-the-chip slab: the
// blockIdx -> slab map keeps each XCD's L2 on its own part of the span (XCD = blockIdx % 8)
template <int U, int T>
__global__ __launch_bounds__(T) void k_unpack_xcd(const v4u *__restrict__ src, v4u *__restrict__ dst, size_t rows) {
    const size_t nb = gridDim.x, per = nb / 8;
    const size_t b = blockIdx.x, slab = (b % 8) * per + b / 8;
    const size_t base = slab * T * U + threadIdx.x;
    v4u v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const size_t u = base + (size_t)k * T;
        if (u < rows) v[k] = __builtin_nontemporal_load(src + u);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const size_t u = base + (size_t)k * T;
        if (u < rows) dst[2 * u] = v[k];
    }
}

// the product kernel's shape with its end-of-workgroup completion (mv2::block_done: stores
// drained, sub-counters, host word), one tile per workgroup (GS = 0) or a fixed grid striding
// over the tiles (GS = grid): the completion's drain is paid once per workgroup
template <int U, int T, bool UNPACK, bool DONE>
__global__ __launch_bounds__(T) void k_units_done(const v4u *__restrict__ src, v4u *__restrict__ dst, size_t rows,
                                                  size_t su, mv2::Done d) {
    const size_t step = (size_t)gridDim.x * T * U;
    for (size_t base = (size_t)blockIdx.x * T * U + threadIdx.x; base < rows; base += step) {
        v4u v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const size_t u = base + (size_t)k * T;
            if (u < rows) v[k] = __builtin_nontemporal_load(src + (UNPACK ? u : u * su));
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const size_t u = base + (size_t)k * T;
            if (u < rows) dst[UNPACK ? u * su : u] = v[k];
        }
    }
    if (DONE) mv2::block_done(d);
}

struct Res {
    const char *name;
    float ms;
    bool ok;
};

int main() {
    const size_t rows = (size_t)8 << 20, su = 2;
    const size_t span = rows * 32, packed = rows * 16;
    std::vector<unsigned> h(span / 4);
    unsigned x = 12345;
    for (auto &v : h) v = (x = x * 1664525u + 1013904223u);
    std::vector<unsigned> want_pack(packed / 4);
    for (size_t i = 0; i < rows; ++i) memcpy(&want_pack[i * 4], &h[i * 8], 16);
    v4u *dspan, *dpack, *dout;
    CK(hipMalloc(&dspan, span));
    CK(hipMalloc(&dpack, packed));
    CK(hipMalloc(&dout, span));
    CK(hipMemcpy(dspan, h.data(), span, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 30;
    std::vector<unsigned> got(span / 4);

    auto time_pack = [&](const char *name, auto launch) -> Res {
        hipMemset(dpack, 0, packed);
        launch();
        hipDeviceSynchronize();
        hipMemcpy(got.data(), dpack, packed, hipMemcpyDeviceToHost);
        bool ok = memcmp(got.data(), want_pack.data(), packed) == 0;
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(e0);
        for (int i = 0; i < iters; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        return Res{name, ms / iters, ok};
    };
    // unpack into a span pre-filled with a sentinel: gap bytes must keep it
    auto time_unpack = [&](const char *name, auto launch) -> Res {
        hipMemset(dout, 0xA5, span);
        (void)hipMemcpy(dpack, want_pack.data(), packed, hipMemcpyHostToDevice);
        launch();
        hipDeviceSynchronize();
        hipMemcpy(got.data(), dout, span, hipMemcpyDeviceToHost);
        bool ok = true;
        for (size_t i = 0; i < rows && ok; ++i) {
            ok = memcmp(&got[i * 8], &h[i * 8], 16) == 0;
            for (int k = 4; k < 8; ++k) ok = ok && got[i * 8 + k] == 0xA5A5A5A5u;
        }
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(e0);
        for (int i = 0; i < iters; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        return Res{name, ms / iters, ok};
    };
    std::vector<Res> rs;
#define PK(U, T, LNT, SNT)                                                                                   \
    rs.push_back(time_pack("pack units U=" #U " T=" #T " lnt=" #LNT " snt=" #SNT, [&] {                   \
        hipLaunchKernelGGL((k_units<U, T, LNT, SNT, false>), dim3((rows + T * U - 1) / (T * U)), dim3(T), 0, 0, \
                           dspan, dpack, rows, su);                                                          \
    }))
#define UK(U, T, LNT, SNT)                                                                                   \
    rs.push_back(time_unpack("unpack units U=" #U " T=" #T " lnt=" #LNT " snt=" #SNT, [&] {               \
        hipLaunchKernelGGL((k_units<U, T, LNT, SNT, true>), dim3((rows + T * U - 1) / (T * U)), dim3(T), 0, 0,  \
                           dpack, dout, rows, su);                                                           \
    }))
    PK(4, 256, true, true);  // the product shape before this sweep
    PK(4, 256, true, false);
    PK(2, 256, true, false);
    PK(8, 256, true, false);
    PK(4, 512, true, false);
    PK(2, 512, true, false);
    PK(8, 512, true, true);
    PK(4, 256, false, false);
    PK(16, 256, true, false);
    for (int g : {1024, 2048, 4096}) {
        char *nm = new char[80];
        snprintf(nm, 80, "pack grid-stride U=4 T=512 grid=%d plain store", g);
        rs.push_back(time_pack(nm, [&] {
            hipLaunchKernelGGL((k_units_gs<4, 512, false, false>), dim3(g), dim3(512), 0, 0, dspan, dpack, rows, su);
        }));
    }
    rs.push_back(time_pack("pack perm2 T=256 plain store", [&] {
        hipLaunchKernelGGL((k_pack_perm2<256, false>), dim3(rows / 256), dim3(256), 0, 0, dspan, dpack, rows);
    }));
    rs.push_back(time_pack("pack perm2 T=256 nt store", [&] {
        hipLaunchKernelGGL((k_pack_perm2<256, true>), dim3(rows / 256), dim3(256), 0, 0, dspan, dpack, rows);
    }));
    UK(4, 256, true, true);  // the product shape before this sweep
    UK(4, 256, true, false);
    UK(8, 256, true, true);
    UK(8, 256, true, false);
    UK(4, 512, true, true);
    UK(2, 512, true, false);
    UK(16, 256, true, true);
    UK(4, 256, false, true);
    for (int g : {1024, 2048, 4096}) {
        char *nm = new char[80];
        snprintf(nm, 80, "unpack grid-stride U=4 T=512 grid=%d nt store", g);
        rs.push_back(time_unpack(nm, [&] {
            hipLaunchKernelGGL((k_units_gs<4, 512, true, true>), dim3(g), dim3(512), 0, 0, dpack, dout, rows, su);
        }));
    }
    UK(2, 256, true, false);
    UK(1, 1024, true, false);
    UK(2, 1024, true, false);
    rs.push_back(time_unpack("unpack xcd-slab U=2 T=512", [&] {
        hipLaunchKernelGGL((k_unpack_xcd<2, 512>), dim3(rows / 1024), dim3(512), 0, 0, dpack, dout, rows);
    }));
    rs.push_back(time_unpack("unpack xcd-slab U=4 T=256", [&] {
        hipLaunchKernelGGL((k_unpack_xcd<4, 256>), dim3(rows / 1024), dim3(256), 0, 0, dpack, dout, rows);
    }));
    // completion-word cost: the product's block_done on the one-tile shape and on fixed grids
    uint32_t *dctr = nullptr;
    uint64_t *dflag = nullptr;
    CK(hipMalloc(&dctr, mv2::kDoneBytes));
    CK(hipMemset(dctr, 0, mv2::kDoneBytes));
    CK(hipHostMalloc((void **)&dflag, 64, hipHostMallocDefault));
    static uint64_t seq = 0;
#define DV(U, T, UNPACK, DONE, GRID)                                                                          \
    do {                                                                                                      \
        char *nm = new char[120];                                                                             \
        const size_t g_ = (GRID) ? (size_t)(GRID) : (rows + (T) * (U) - 1) / ((T) * (U));                     \
        snprintf(nm, 120, "%s %s U=%d T=%d grid=%zu", UNPACK ? "unpack" : "pack", DONE ? "done" : "nodone", U, T, g_); \
        auto fn = [&] {                                                                                       \
            mv2::Done d_{dctr, dflag, ++seq};                                                                 \
            hipLaunchKernelGGL((k_units_done<U, T, UNPACK, DONE>), dim3(g_), dim3(T), 0, 0,                   \
                               UNPACK ? dpack : dspan, UNPACK ? dout : dpack, rows, su, d_);                  \
        };                                                                                                    \
        rs.push_back(UNPACK ? time_unpack(nm, fn) : time_pack(nm, fn));                                       \
    } while (0)
    DV(2, 512, true, false, 0);
    DV(2, 512, true, true, 0);
    DV(1, 1024, true, true, 0);
    DV(2, 512, false, false, 0);
    DV(2, 512, false, true, 0);
    for (int g : {512, 1024, 2048, 4096}) {
        DV(2, 512, true, true, g);
        DV(2, 1024, true, true, g);
        DV(4, 512, true, true, g);
        DV(2, 512, false, true, g);
        DV(4, 512, false, true, g);
    }
    // MPI_Pack then MPI_Unpack of the same buffers back to back (the pack_overhead probe's
    // sequence): the pair's time, to compare with the two kernels timed apart
    rs.push_back(time_pack("pair: pack + unpack alternating (ms per pair)", [&] {
        mv2::Done d_{dctr, dflag, ++seq};
        hipLaunchKernelGGL((k_units_done<2, 512, false, true>), dim3(rows / 1024), dim3(512), 0, 0, dspan, dpack, rows, su, d_);
        mv2::Done e_{dctr, dflag, ++seq};
        hipLaunchKernelGGL((k_units_done<2, 512, true, true>), dim3(rows / 1024), dim3(512), 0, 0, dpack, dspan, rows, su, e_);
    }));
    // write-only / whole-sector references (traffic floors of the unpack's write side)
    rs.push_back(time_pack("ref: write-only 256 MiB whole lines", [&] {
        hipLaunchKernelGGL((k_write_only<512, false>), dim3(span / 16 / 512), dim3(512), 0, 0, dout, span / 16);
    }));
    rs.push_back(time_pack("ref: write-only 16 of every 32 bytes over 256 MiB", [&] {
        hipLaunchKernelGGL((k_write_only<512, true>), dim3(rows / 512), dim3(512), 0, 0, dout, rows);
    }));
    rs.push_back(time_pack("ref: read 128 MiB + write 256 MiB whole sectors (gap overwritten)", [&] {
        hipLaunchKernelGGL((k_expand_whole<512>), dim3(rows / 512), dim3(512), 0, 0, dpack, dout, rows);
    }));
    // references: contiguous copy of the span and of the packed bytes
    rs.push_back(time_pack("ref: copy 128 MiB contiguous (packed size)", [&] {
        hipMemcpyAsync(dpack, dspan, packed, hipMemcpyDeviceToDevice, 0);
    }));
    for (auto &r : rs) {
        const bool unpack = !strncmp(r.name, "unpack", 6);
        double floor_b = unpack ? (double)packed + span : (double)span + packed;
        if (!strncmp(r.name, "ref: write-only", 15)) floor_b = (double)span;
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps_algorithmic\": %.1f, \"GBps_hbm_floor\": %.1f, \"ok\": %s}\n",
               r.name, r.ms, 2.0 * packed / (r.ms * 1e6), floor_b / (r.ms * 1e6), r.ok ? "true" : "false");
    }
    return 0;
}
