/* pack_overhead.c — where the host time of a blocking MPI_Pack / MPI_Unpack goes (VERDICT r02
 * weak #4): the configs[4] vector MPI_Type_vector(8Mi, 4, 8, MPI_FLOAT) on device buffers, timed
 * per call through the MPI layer, through the C-ABI strided entry (mv2h_*_strided, no datatype
 * lookup) and, for scale, MPI_Reduce_local on 256 MiB and hipPointerGetAttributes alone.
 * Prints one JSON line. */
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <mv2h.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

/* random bytes, not zeros: zero-filled operands stream faster than real data on this GPU */
static void fill_random(void *d, size_t bytes) {
    unsigned *h = (unsigned *)malloc(bytes);
    unsigned x = 12345;
    for (size_t i = 0; i < bytes / 4; ++i) h[i] = (x = x * 1664525u + 1013904223u) & 0x3f7fffffu;
    hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    free(h);
}

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

#define REPS 50

int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    const int nb = 8 << 20;
    const size_t span = ((size_t)(nb - 1) * 8 + 4) * 4, packed = (size_t)nb * 16;
    void *src = NULL, *dst = NULL, *a = NULL, *b = NULL;
    hipMalloc(&src, span);
    hipMalloc(&dst, packed);
    fill_random(src, span);
    fill_random(dst, packed);
    MPI_Datatype vt;
    MPI_Type_vector(nb, 4, 8, MPI_FLOAT, &vt);
    MPI_Type_commit(&vt);
    double t_pack = 0, t_unpack = 0, t_cpack = 0, t_cunpack = 0, t_rl = 0, t_attr = 0;
    for (int it = -3; it < REPS; ++it) {
        int pos = 0;
        double t0 = now_us();
        MPI_Pack(src, 1, vt, dst, (int)packed, &pos, MPI_COMM_WORLD);
        double t1 = now_us();
        pos = 0;
        MPI_Unpack(dst, (int)packed, &pos, src, 1, vt, MPI_COMM_WORLD);
        double t2 = now_us();
        mv2h_pack_strided(src, dst, nb, 16, 32, NULL);
        double t3 = now_us();
        mv2h_unpack_strided(dst, src, nb, 16, 32, NULL);
        double t4 = now_us();
        if (it >= 0) {
            t_pack += t1 - t0;
            t_unpack += t2 - t1;
            t_cpack += t3 - t2;
            t_cunpack += t4 - t3;
        }
    }
    const size_t rl = (size_t)64 << 20;
    hipMalloc(&a, rl * 4);
    hipMalloc(&b, rl * 4);
    fill_random(a, rl * 4);
    fill_random(b, rl * 4);
    for (int it = -3; it < REPS; ++it) {
        double t0 = now_us();
        MPI_Reduce_local(a, b, (int)rl, MPI_FLOAT, MPI_SUM);
        double t1 = now_us();
        hipPointerAttribute_t at;
        hipPointerGetAttributes(&at, a);
        double t2 = now_us();
        if (it >= 0) {
            t_rl += t1 - t0;
            t_attr += t2 - t1;
        }
    }
    mv2h_timing_enable(1);
    double k_unpack = 0, k_pack = 0, k_rl = 0;
    for (int it = 0; it < 10; ++it) {
        int pos = 0;
        MPI_Pack(src, 1, vt, dst, (int)packed, &pos, MPI_COMM_WORLD);
        k_pack += mv2h_last_kernel_ms();
        pos = 0;
        MPI_Unpack(dst, (int)packed, &pos, src, 1, vt, MPI_COMM_WORLD);
        k_unpack += mv2h_last_kernel_ms();
        MPI_Reduce_local(a, b, (int)rl, MPI_FLOAT, MPI_SUM);
        k_rl += mv2h_last_kernel_ms();
    }
    mv2h_timing_enable(0);
    printf("{\"mpi_pack_us\": %.2f, \"mpi_unpack_us\": %.2f, \"cabi_pack_strided_us\": %.2f, "
           "\"cabi_unpack_strided_us\": %.2f, \"reduce_local_us\": %.2f, \"hipPointerGetAttributes_us\": %.3f, "
           "\"kernel_pack_us\": %.2f, \"kernel_unpack_us\": %.2f, \"kernel_reduce_local_us\": %.2f}\n",
           t_pack / REPS, t_unpack / REPS, t_cpack / REPS, t_cunpack / REPS, t_rl / REPS, t_attr / REPS,
           k_pack * 100, k_unpack * 100, k_rl * 100);
    MPI_Type_free(&vt);
    MPI_Finalize();
    return 0;
}
