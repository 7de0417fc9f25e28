// pack.hip — strided pack / unpack for MPI_Type_vector-family datatypes.
//
// Replaces the reference's device pack path (MPID_Segment_pack_device
// ibv_cuda_util.c:623 -> cudaMemcpy2DAsync, and pack_unpack_vector_kernel
// pack_unpack.cu:374-481).  Layout: nblocks rows of blk bytes, row i at
// src + i*stride (pack) / dst + i*stride (unpack); packed rows are dense.
//
// Two kernels:
//  * k_pack_units: one thread per g-byte unit (g = widest of 16/8/4/2/1 that
//    divides blk, stride and both base addresses): packed side coalesced,
//    strided side coalesced within a row.
//  * k_pack_lds: rows narrower than 16 bytes with stride <= 64 bytes.  A
//    workgroup loads the whole strided span of its rows into LDS with 16-byte
//    coalesced loads, then assembles 16 packed bytes per thread from LDS and
//    writes them with one 16-byte store.  This is the LDS-staged gather.
#include <hip/hip_runtime.h>

#include "../coll/kernels.h"
#include "../common.h"

namespace mv2 {

template <typename G>
__global__ __launch_bounds__(kThreads) void k_pack_units(const char *__restrict__ src, char *__restrict__ dst,
                                                         size_t nrows, uint32_t upr, size_t stride_units,
                                                         int unpack) {
    const size_t total = nrows * upr;
    const size_t step = (size_t)gridDim.x * kThreads;
    const G *s = (const G *)src;
    G *d = (G *)dst;
    for (size_t u = (size_t)blockIdx.x * kThreads + threadIdx.x; u < total; u += step) {
        const size_t i = u / upr, j = u - i * upr;
        if (!unpack) d[u] = s[i * stride_units + j];
        else d[i * stride_units + j] = s[u];
    }
}

// LDS-staged pack of narrow rows: rows [r0, r0+R) per workgroup.
constexpr int kLdsSpan = 32768;  // bytes of strided span staged per workgroup
__global__ __launch_bounds__(kThreads) void k_pack_lds(const char *__restrict__ src, char *__restrict__ dst,
                                                       size_t nrows, uint32_t blk, uint32_t stride,
                                                       uint32_t rows_per_wg) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const size_t r0 = (size_t)blockIdx.x * rows_per_wg;
    if (r0 >= nrows) return;
    const size_t r1 = r0 + rows_per_wg < nrows ? r0 + rows_per_wg : nrows;
    // strided span [r0*stride, (r1-1)*stride + blk) loaded with 16B vectors from a 16B-aligned base
    const uintptr_t sb = (uintptr_t)src + r0 * stride;
    const uintptr_t se = (uintptr_t)src + (r1 - 1) * stride + blk;
    const uintptr_t ab = sb & ~(uintptr_t)15;
    const uintptr_t ae = (se + 15) & ~(uintptr_t)15;
    const uint32_t nv = (uint32_t)((ae - ab) / 16);
    const v4u *sv = (const v4u *)ab;
    for (uint32_t v = threadIdx.x; v < nv; v += kThreads) ((v4u *)lds)[v] = sv[v];
    __syncthreads();
    const uint32_t lead = (uint32_t)(sb - ab);
    const size_t out_bytes = (r1 - r0) * blk;
    char *o = dst + r0 * blk;
    size_t done = 0;
    if ((uintptr_t)o % 16 == 0) {
        // 16 packed bytes per thread: byte reads from LDS, one 16-byte store
        const size_t nch = out_bytes / 16;
        for (size_t c = threadIdx.x; c < nch; c += kThreads) {
            union { v4u v; char b[16]; } u;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t b = (uint32_t)(c * 16 + k);
                const uint32_t row = b / blk, col = b - row * blk;
                u.b[k] = lds[lead + row * stride + col];
            }
            st_nt((v4u *)o + c, u.v);
        }
        done = nch * 16;
    }
    for (size_t b = done + threadIdx.x; b < out_bytes; b += kThreads) {
        const uint32_t row = (uint32_t)(b / blk), col = (uint32_t)(b - (size_t)row * blk);
        o[b] = lds[lead + row * stride + col];
    }
}

int launch_pack_strided(const void *src, void *dst, size_t nblocks, size_t blk, size_t stride, int unpack,
                        hipStream_t stream) {
    if (nblocks == 0 || blk == 0) return 0;
    if (!unpack && blk < 16 && stride <= 64 && stride >= blk) {
        const uint32_t rows = (uint32_t)((kLdsSpan - 32) / stride);
        const size_t g = (nblocks + rows - 1) / rows;
        hipLaunchKernelGGL(k_pack_lds, dim3(g), dim3(kThreads), kLdsSpan, stream, (const char *)src, (char *)dst,
                           nblocks, (uint32_t)blk, (uint32_t)stride, rows);
        return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
    }
    size_t g = 16;
    const uintptr_t a = (uintptr_t)src | (uintptr_t)dst;
    while (g > 1 && ((blk % g) || (stride % g) || (a % g))) g >>= 1;
    const size_t upr = blk / g;
    const size_t total = nblocks * upr;
    size_t grid = (total + kThreads - 1) / kThreads;
    if (grid > 4096) grid = 4096;
    const size_t su = stride / g;
    switch (g) {
    case 16: hipLaunchKernelGGL(k_pack_units<v4u>, dim3(grid), dim3(kThreads), 0, stream, (const char *)src, (char *)dst, nblocks, (uint32_t)upr, su, unpack); break;
    case 8: hipLaunchKernelGGL(k_pack_units<uint64_t>, dim3(grid), dim3(kThreads), 0, stream, (const char *)src, (char *)dst, nblocks, (uint32_t)upr, su, unpack); break;
    case 4: hipLaunchKernelGGL(k_pack_units<uint32_t>, dim3(grid), dim3(kThreads), 0, stream, (const char *)src, (char *)dst, nblocks, (uint32_t)upr, su, unpack); break;
    case 2: hipLaunchKernelGGL(k_pack_units<uint16_t>, dim3(grid), dim3(kThreads), 0, stream, (const char *)src, (char *)dst, nblocks, (uint32_t)upr, su, unpack); break;
    default: hipLaunchKernelGGL(k_pack_units<uint8_t>, dim3(grid), dim3(kThreads), 0, stream, (const char *)src, (char *)dst, nblocks, (uint32_t)upr, su, unpack); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
}

}  // namespace mv2
