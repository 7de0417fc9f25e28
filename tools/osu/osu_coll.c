/*
 * osu_coll.c — OSU-micro-benchmark-compatible collective timing loop written
 * against the drop-in include/mpi.h and linked with mvapich2_amd's libmpi.so.
 * Same measurement loop as the reference harness (osu_allreduce.c:98-163:
 * per size, skip warmup iterations, then Barrier; t0; collective; t1; sum;
 * report the average over ranks of per-rank mean latency), with `-d rocm`
 * device buffers and busbw columns added (OMB prints latency only).
 *
 *   osu_coll -c allreduce|reduce|reduce_scatter|allgather|bcast|reduce_local|latency|bw|all
 *            [-m min:max bytes] [-f size factor (2)] [-i iters] [-I large-message iters]
 *            [-x warmup] [-C cap bytes for -c all's reduce_scatter/allgather/bcast]
 *            [-d rocm|host] [-v (validate every collective)] [-j (JSON rows)]
 * -c all runs allreduce over [min, max] and reduce_scatter, allgather, bcast over
 * [min, min(max, cap)] in one job (bench.py's N > 1 sweep: configs[2] and [3]), then the
 * device point-to-point latency and bandwidth between ranks 0 and 1 up to 16 MiB.
 */
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const char *coll = "allreduce";
static size_t min_sz = 8, max_sz = 1 << 20, cap_sz = (size_t)256 << 20, factor = 2;
static int iters_small = 1000, iters_large = 100, skip_small = 100, skip_large = 10;
static int device = 1, validate = 0, json = 0;
static FILE *jout = NULL; /* JSON rows: stdout, or the -o file (rank 0) */

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
static int run_pt2pt(int rank, void *sbuf, void *rbuf, size_t lo, size_t hi) {
    const int window = 64;
    MPI_Request reqs[64];
    for (size_t sz = lo; sz <= hi; sz *= factor) {
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
        if (rank == 0 && json) {
            if (!strcmp(coll, "latency"))
                fprintf(jout, "JSON {\"coll\": \"osu_latency\", \"bytes\": %zu, \"lat_us\": %.2f, \"iters\": %d}\n", sz,
                       t / iters / 2 * 1e6, iters);
            else
                fprintf(jout, "JSON {\"coll\": \"osu_bw\", \"bytes\": %zu, \"bw_GBps\": %.3f, \"iters\": %d}\n", sz,
                       (double)sz * window * iters / t / 1e9, iters);
            fflush(jout);
        } else if (rank == 0) {
            if (!strcmp(coll, "latency")) printf("%-12zu %14.2f\n", sz, t / iters / 2 * 1e6);
            else printf("%-12zu %14.2f\n", sz, (double)sz * window * iters / t / 1e9);
        }
    }
    return 0;
}

/* result check of one collective (-v): every element against its closed form for the OMB fill
 * (i % 100 + 1) * (rank + 1); returns 1 when right */
static int check(const char *c, const void *rbuf, size_t count, size_t sz, int rank, int size, const int *counts) {
    if (!strcmp(c, "reduce") || !strcmp(c, "reduce_local")) return 1;
    size_t n = !strcmp(c, "allgather") ? sz * (size_t)size : !strcmp(c, "bcast") ? sz : count * sizeof(float);
    if (!strcmp(c, "reduce_scatter")) n = (size_t)counts[rank] * sizeof(float);
    char *h = (char *)malloc(n ? n : 1);
    if (device) hipMemcpy(h, !strcmp(c, "bcast") ? rbuf : rbuf, n, hipMemcpyDeviceToHost);
    else memcpy(h, rbuf, n);
    int ok = 1;
    const float tot = (float)(size * (size + 1) / 2);
    if (!strcmp(c, "allreduce")) {
        const float *f = (const float *)h;
        for (size_t i = 0; i < count && ok; ++i) ok = f[i] == (float)(i % 100 + 1) * tot;
    } else if (!strcmp(c, "reduce_scatter")) {
        size_t off = 0;
        for (int r = 0; r < rank; ++r) off += (size_t)counts[r];
        const float *f = (const float *)h;
        for (size_t i = 0; i < (size_t)counts[rank] && ok; ++i) ok = f[i] == (float)((off + i) % 100 + 1) * tot;
    } else {
        /* allgather: block j = rank j's first sz bytes of its fill; bcast: rank 0's (bytes of floats) */
        float *want = (float *)malloc((sz / 4 + 1) * sizeof(float));
        for (int j = 0; j < (!strcmp(c, "allgather") ? size : 1) && ok; ++j) {
            for (size_t i = 0; i < sz / 4 + 1; ++i) want[i] = (float)((i % 100 + 1) * (j + 1));
            ok = memcmp(h + (size_t)j * sz, want, sz) == 0;
        }
        free(want);
    }
    free(h);
    return ok;
}

static int run_coll(const char *c, int rank, int size, void *sbuf, void *rbuf, size_t lo, size_t hi) {
    if (rank == 0 && !json) {
        printf("# mvapich2_amd osu_coll -c %s, %d ranks, %s buffers\n", c, size, device ? "ROCm device" : "host");
        printf("%-12s %14s %14s %14s %12s\n", "# Size(B)", "Avg Lat(us)", "algbw(GB/s)", "busbw(GB/s)", "valid");
    }
    int *counts = (int *)malloc(sizeof(int) * size);
    int bad_any = 0;
    for (size_t sz = lo; sz <= hi; sz *= factor) {
        const size_t count = sz / sizeof(float) ? sz / sizeof(float) : 1;
        const int large = count > 8192; /* osu_allreduce.c:101 */
        const int iters = large ? iters_large : iters_small, skip = large ? skip_large : skip_small;
        /* the fill covers what allgather / bcast send (sz bytes) and the reducing operands */
        fill(sbuf, (sz + 3) / 4 > count ? (sz + 3) / 4 : count, rank);
        if (!strcmp(c, "bcast") && rank != 0) {
            if (device) hipMemset(sbuf, 0xA5, sz);
            else memset(sbuf, 0xA5, sz);
        }
        double total = 0.0;
        int rc = 0;
        {
            int base = (int)(count / size), rem = (int)(count % size);
            for (int r = 0; r < size; ++r) counts[r] = base + (r < rem);
        }
        for (int it = 0; it < iters + skip; ++it) {
            MPI_Barrier(MPI_COMM_WORLD);
            double t0 = MPI_Wtime();
            if (!strcmp(c, "allreduce")) rc |= MPI_Allreduce(sbuf, rbuf, (int)count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
            else if (!strcmp(c, "reduce")) rc |= MPI_Reduce(sbuf, rbuf, (int)count, MPI_FLOAT, MPI_SUM, 0, MPI_COMM_WORLD);
            else if (!strcmp(c, "reduce_local")) rc |= MPI_Reduce_local(sbuf, rbuf, (int)count, MPI_FLOAT, MPI_SUM);
            /* osu_reduce_scatter.c:116-131: size/n each, first size%n ranks one more */
            else if (!strcmp(c, "reduce_scatter")) rc |= MPI_Reduce_scatter(sbuf, rbuf, counts, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
            else if (!strcmp(c, "allgather")) rc |= MPI_Allgather(sbuf, (int)sz, MPI_CHAR, rbuf, (int)sz, MPI_CHAR, MPI_COMM_WORLD);
            else if (!strcmp(c, "bcast")) rc |= MPI_Bcast(sbuf, (int)sz, MPI_CHAR, 0, MPI_COMM_WORLD);
            double t1 = MPI_Wtime();
            if (it >= skip) total += t1 - t0;
        }
        double lat = total / iters * 1e6, sum = 0.0;
        MPI_Allreduce(MPI_IN_PLACE, &lat, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
        sum = lat / size;
        int valid = 1;
        if (validate) {
            int mine = check(c, !strcmp(c, "bcast") ? sbuf : rbuf, count, sz, rank, size, counts), all = 0;
            MPI_Allreduce(&mine, &all, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
            valid = all == size;
        }
        double algbw = sz / (sum * 1e-6) / 1e9;
        double bf = 1.0;
        if (!strcmp(c, "allreduce")) bf = 2.0 * (size - 1) / size;
        else if (!strcmp(c, "reduce_scatter") || !strcmp(c, "allgather")) bf = (double)(size - 1) / size;
        if (!strcmp(c, "allgather")) algbw *= size;
        if (!strcmp(c, "reduce_local")) { bf = 3.0; }
        bad_any |= rc || (validate && !valid);
        if (rank == 0 && json)
            fprintf(jout, "JSON {\"coll\": \"%s\", \"bytes\": %zu, \"lat_us\": %.2f, \"algbw_GBps\": %.3f, \"busbw_GBps\": %.3f, "
                   "\"iters\": %d, \"valid\": %s}\n", c, sz, sum, algbw, algbw * bf, iters,
                   rc ? "false" : (validate ? (valid ? "true" : "false") : "null"));
        else if (rank == 0)
            printf("%-12zu %14.2f %14.2f %14.2f %12s\n", sz, sum, algbw, algbw * bf,
                   rc ? "ERROR" : (validate ? (valid ? "ok" : "WRONG") : "-"));
        if (rank == 0) fflush(json ? jout : stdout);
    }
    free(counts);
    return bad_any;
}

/* The whole program.  init = 0: MPI is already initialised by the caller (bench.py loads this file
 * as libosu_coll.so into its ranks and calls osu_coll_main: the sweep then runs in the bench's
 * own MPI job, on its tuning, with no second process per GPU); MPI_Finalize is left to it too. */
static int osu_run(int argc, char **argv, int init) {
    /* defaults again: the library entry may be called more than once */
    coll = "allreduce";
    min_sz = 8, max_sz = 1 << 20, cap_sz = (size_t)256 << 20, factor = 2;
    iters_small = 1000, iters_large = 100, skip_small = 100, skip_large = 10;
    device = 1, validate = 0, json = 0;
    const char *jpath = NULL;
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
        else if (!strcmp(argv[i], "-I") && i + 1 < argc) iters_large = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-f") && i + 1 < argc) factor = strtoull(argv[++i], NULL, 10);
        else if (!strcmp(argv[i], "-C") && i + 1 < argc) cap_sz = strtoull(argv[++i], NULL, 10);
        else if (!strcmp(argv[i], "-j")) json = 1;
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) jpath = argv[++i];
        else { fprintf(stderr, "osu_coll: unknown argument %s\n", argv[i]); return 2; }
    }
    if (init) MPI_Init(&argc, &argv);
    int rank, size;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    jout = stdout;
    if (json && jpath && rank == 0 && !(jout = fopen(jpath, "w"))) {
        fprintf(stderr, "osu_coll: cannot write %s\n", jpath);
        jout = stdout;
    }
    const size_t gather_max = (!strcmp(coll, "all") ? (max_sz < cap_sz ? max_sz : cap_sz) : max_sz) * (size_t)size;
    const size_t maxb = gather_max > max_sz ? gather_max : max_sz;
    void *sbuf = alloc_buf(maxb), *rbuf = alloc_buf(maxb);
    if (!sbuf || !rbuf) { fprintf(stderr, "allocation failed\n"); MPI_Abort(MPI_COMM_WORLD, 1); }
    if (!strcmp(coll, "latency") || !strcmp(coll, "bw")) {
        if (size < 2) { fprintf(stderr, "-c %s needs 2 ranks\n", coll); MPI_Abort(MPI_COMM_WORLD, 1); }
        if (rank == 0)
            printf("# mvapich2_amd osu_%s (pt2pt, ranks 0 <-> 1), %s buffers\n%-12s %14s\n", coll,
                   device ? "ROCm device" : "host", "# Size(B)", !strcmp(coll, "latency") ? "Latency(us)" : "BW(GB/s)");
        run_pt2pt(rank, sbuf, rbuf, min_sz, max_sz);
        if (device) {
            hipFree(sbuf);
            hipFree(rbuf);
        } else {
            free(sbuf);
            free(rbuf);
        }
        if (init) MPI_Finalize();
        return 0;
    }
    if (factor < 2) factor = 2;
    int rc = 0;
    if (!strcmp(coll, "all")) {
        static const char *const all[4] = {"allreduce", "reduce_scatter", "allgather", "bcast"};
        for (int k = 0; k < 4 && !rc; ++k)
            rc = run_coll(all[k], rank, size, sbuf, rbuf, min_sz, k ? (max_sz < cap_sz ? max_sz : cap_sz) : max_sz);
        /* device point-to-point, ranks 0 <-> 1 (osu_latency.c / osu_bw.c patterns) up to 16 MiB */
        const size_t p2p_hi = max_sz < ((size_t)16 << 20) ? max_sz : ((size_t)16 << 20);
        if (!rc && size >= 2) {
            coll = "latency";
            rc = run_pt2pt(rank, sbuf, rbuf, min_sz, p2p_hi);
            coll = "bw";
            if (!rc) rc = run_pt2pt(rank, sbuf, rbuf, min_sz, p2p_hi);
        }
    } else {
        rc = run_coll(coll, rank, size, sbuf, rbuf, min_sz, max_sz);
    }
    if (device) {
        hipFree(sbuf);
        hipFree(rbuf);
    } else {
        free(sbuf);
        free(rbuf);
    }
    if (jout && jout != stdout) fclose(jout);
    jout = NULL;
    if (init) MPI_Finalize();
    return rc;
}

#ifdef OSU_COLL_LIB
int osu_coll_main(int argc, char **argv) { return osu_run(argc, argv, 0); }
#else
int main(int argc, char **argv) { return osu_run(argc, argv, 1); }
#endif
