/*
 * osu_coll.c — OSU-micro-benchmark-compatible collective timing loop written
 * against the drop-in include/mpi.h and linked with mvapich2_amd's libmpi.so.
 * Same measurement loop as the reference harness (osu_allreduce.c:98-163:
 * per size, skip warmup iterations, then Barrier; t0; collective; t1; sum;
 * report the average over ranks of per-rank mean latency), with `-d rocm`
 * device buffers and busbw columns added (OMB prints latency only).
 *
 *   osu_coll -c allreduce|reduce|reduce_scatter|allgather|bcast|reduce_local|latency|bw
 *            [-m min:max bytes] [-i iters] [-x warmup] [-d rocm|host] [-v]
 */
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const char *coll = "allreduce";
static size_t min_sz = 8, max_sz = 1 << 20;
static int iters_small = 1000, iters_large = 100, skip_small = 100, skip_large = 10;
static int device = 1, validate = 0;

static void *alloc_buf(size_t bytes) {
    void *p = NULL;
    if (device) {
        if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) return NULL;
        hipMemset(p, 0, bytes ? bytes : 1);
    } else {
        p = calloc(1, bytes ? bytes : 1);
    }
    return p;
}

static void fill(void *p, size_t count, int rank) {
    float *h = (float *)malloc(count * sizeof(float));
    for (size_t i = 0; i < count; ++i) h[i] = (float)((i % 100 + 1) * (rank + 1)); /* OMB pattern */
    if (device) hipMemcpy(p, h, count * sizeof(float), hipMemcpyHostToDevice);
    else memcpy(p, h, count * sizeof(float));
    free(h);
}

/* osu_latency / osu_bw patterns between ranks 0 and 1 (osu_latency.c, osu_bw.c):
 * latency = half the ping-pong round trip; bw = a window of 64 Isend/Irecv then
 * the receiver's 4-byte ack, bytes / time. */
static int run_pt2pt(int rank, void *sbuf, void *rbuf) {
    const int window = 64;
    MPI_Request reqs[64];
    for (size_t sz = min_sz; sz <= max_sz; sz *= 2) {
        const int large = sz > 8192;
        const int iters = large ? iters_large : iters_small, skip = large ? skip_large : skip_small;
        double t0 = 0.0;
        MPI_Barrier(MPI_COMM_WORLD);
        for (int it = 0; it < iters + skip; ++it) {
            if (it == skip) t0 = MPI_Wtime();
            if (!strcmp(coll, "latency")) {
                if (rank == 0) {
                    MPI_Send(sbuf, (int)sz, MPI_CHAR, 1, 1, MPI_COMM_WORLD);
                    MPI_Recv(rbuf, (int)sz, MPI_CHAR, 1, 1, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
                } else if (rank == 1) {
                    MPI_Recv(rbuf, (int)sz, MPI_CHAR, 0, 1, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
                    MPI_Send(sbuf, (int)sz, MPI_CHAR, 0, 1, MPI_COMM_WORLD);
                }
            } else {
                if (rank == 0) {
                    for (int w = 0; w < window; ++w) MPI_Isend(sbuf, (int)sz, MPI_CHAR, 1, 100, MPI_COMM_WORLD, &reqs[w]);
                    MPI_Waitall(window, reqs, MPI_STATUSES_IGNORE);
                    MPI_Recv(rbuf, 4, MPI_CHAR, 1, 101, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
                } else if (rank == 1) {
                    for (int w = 0; w < window; ++w) MPI_Irecv(rbuf, (int)sz, MPI_CHAR, 0, 100, MPI_COMM_WORLD, &reqs[w]);
                    MPI_Waitall(window, reqs, MPI_STATUSES_IGNORE);
                    MPI_Send(sbuf, 4, MPI_CHAR, 0, 101, MPI_COMM_WORLD);
                }
            }
        }
        const double t = MPI_Wtime() - t0;
        if (rank == 0) {
            if (!strcmp(coll, "latency")) printf("%-12zu %14.2f\n", sz, t / iters / 2 * 1e6);
            else printf("%-12zu %14.2f\n", sz, (double)sz * window * iters / t / 1e9);
        }
    }
    return 0;
}

int main(int argc, char **argv) {
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-c") && i + 1 < argc) coll = argv[++i];
        else if (!strcmp(argv[i], "-m") && i + 1 < argc) {
            char *c = strchr(argv[++i], ':');
            if (c) { *c = 0; min_sz = strtoull(argv[i], NULL, 10); max_sz = strtoull(c + 1, NULL, 10); }
            else max_sz = strtoull(argv[i], NULL, 10);
        } else if (!strcmp(argv[i], "-i") && i + 1 < argc) iters_small = iters_large = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-x") && i + 1 < argc) skip_small = skip_large = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-d") && i + 1 < argc) device = strcmp(argv[++i], "host") != 0;
        else if (!strcmp(argv[i], "-v")) validate = 1;
    }
    MPI_Init(&argc, &argv);
    int rank, size;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    const size_t maxb = max_sz * (size_t)size;
    void *sbuf = alloc_buf(maxb), *rbuf = alloc_buf(maxb);
    if (!sbuf || !rbuf) { fprintf(stderr, "allocation failed\n"); MPI_Abort(MPI_COMM_WORLD, 1); }
    if (!strcmp(coll, "latency") || !strcmp(coll, "bw")) {
        if (size < 2) { fprintf(stderr, "-c %s needs 2 ranks\n", coll); MPI_Abort(MPI_COMM_WORLD, 1); }
        if (rank == 0)
            printf("# mvapich2_amd osu_%s (pt2pt, ranks 0 <-> 1), %s buffers\n%-12s %14s\n", coll,
                   device ? "ROCm device" : "host", "# Size(B)", !strcmp(coll, "latency") ? "Latency(us)" : "BW(GB/s)");
        run_pt2pt(rank, sbuf, rbuf);
        MPI_Finalize();
        return 0;
    }
    if (rank == 0) {
        printf("# mvapich2_amd osu_coll -c %s, %d ranks, %s buffers\n", coll, size, device ? "ROCm device" : "host");
        printf("%-12s %14s %14s %14s %12s\n", "# Size(B)", "Avg Lat(us)", "algbw(GB/s)", "busbw(GB/s)", "valid");
    }
    int *counts = (int *)malloc(sizeof(int) * size);
    for (size_t sz = min_sz; sz <= max_sz; sz *= 2) {
        const size_t count = sz / sizeof(float) ? sz / sizeof(float) : 1;
        const int large = count > 8192; /* osu_allreduce.c:101 */
        const int iters = large ? iters_large : iters_small, skip = large ? skip_large : skip_small;
        fill(sbuf, count, rank);
        double total = 0.0;
        int rc = 0;
        for (int it = 0; it < iters + skip; ++it) {
            MPI_Barrier(MPI_COMM_WORLD);
            double t0 = MPI_Wtime();
            if (!strcmp(coll, "allreduce")) rc |= MPI_Allreduce(sbuf, rbuf, (int)count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
            else if (!strcmp(coll, "reduce")) rc |= MPI_Reduce(sbuf, rbuf, (int)count, MPI_FLOAT, MPI_SUM, 0, MPI_COMM_WORLD);
            else if (!strcmp(coll, "reduce_local")) rc |= MPI_Reduce_local(sbuf, rbuf, (int)count, MPI_FLOAT, MPI_SUM);
            else if (!strcmp(coll, "reduce_scatter")) {
                /* osu_reduce_scatter.c:116-131: size/n each, first size%n ranks one more */
                int base = (int)(count / size), rem = (int)(count % size);
                for (int r = 0; r < size; ++r) counts[r] = base + (r < rem);
                rc |= MPI_Reduce_scatter(sbuf, rbuf, counts, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
            } else if (!strcmp(coll, "allgather")) rc |= MPI_Allgather(sbuf, (int)sz, MPI_CHAR, rbuf, (int)sz, MPI_CHAR, MPI_COMM_WORLD);
            else if (!strcmp(coll, "bcast")) rc |= MPI_Bcast(sbuf, (int)sz, MPI_CHAR, 0, MPI_COMM_WORLD);
            double t1 = MPI_Wtime();
            if (it >= skip) total += t1 - t0;
        }
        double lat = total / iters * 1e6, sum = 0.0;
        MPI_Allreduce(device ? MPI_IN_PLACE : MPI_IN_PLACE, &lat, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
        sum = lat / size;
        int valid = 1;
        if (validate && !strcmp(coll, "allreduce")) {
            float *h = (float *)malloc(count * sizeof(float));
            if (device) hipMemcpy(h, rbuf, count * sizeof(float), hipMemcpyDeviceToHost);
            else memcpy(h, rbuf, count * sizeof(float));
            for (size_t i = 0; i < count && valid; ++i) {
                float want = (float)((i % 100 + 1) * (size * (size + 1) / 2));
                if (h[i] != want) valid = 0;
            }
            free(h);
        }
        double algbw = sz / (sum * 1e-6) / 1e9;
        double factor = 1.0;
        if (!strcmp(coll, "allreduce")) factor = 2.0 * (size - 1) / size;
        else if (!strcmp(coll, "reduce_scatter") || !strcmp(coll, "allgather")) factor = (double)(size - 1) / size;
        if (!strcmp(coll, "allgather")) algbw *= size;
        if (!strcmp(coll, "reduce_local")) { factor = 3.0; }
        if (rank == 0)
            printf("%-12zu %14.2f %14.2f %14.2f %12s\n", sz, sum, algbw, algbw * factor,
                   rc ? "ERROR" : (validate ? (valid ? "ok" : "WRONG") : "-"));
    }
    free(counts);
    MPI_Finalize();
    return 0;
}
