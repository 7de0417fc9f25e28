/* uop_vsum.c — the configs[4] user op of bench.py as a C MPI_User_function (an application's op
 * is C in the reference's OSU suite): inout += in on the type map of MPI_Type_vector(nb, 4, 8,
 * MPI_FLOAT) elements, nb set by uop_vsum_blocks().  Built into libuop_vsum.so. */
#include <mpi.h>

static long g_nb = 1;

void uop_vsum_blocks(long nb) { g_nb = nb; }

void uop_vsum(void *in, void *inout, int *len, MPI_Datatype *dt) {
    (void)dt;
    const long ext = (g_nb - 1) * 8 + 4; /* floats per element extent */
    const float *a = (const float *)in;
    float *b = (float *)inout;
    for (long e = 0; e < *len; ++e)
        for (long i = 0; i < g_nb; ++i) {
            const long o = e * ext + i * 8;
            b[o] += a[o];
            b[o + 1] += a[o + 1];
            b[o + 2] += a[o + 2];
            b[o + 3] += a[o + 3];
        }
}
