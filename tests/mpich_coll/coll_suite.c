/* coll_suite.c — the reference's own collective tests (MPICH test/mpi/coll, shipped with
 * MVAPICH2 2.3.7), restated as one self-checking C program linked against the drop-in
 * libmpi.so: the same operations, operands, user functions and expected values as each test
 * program, on MPI_COMM_WORLD (the reference iterates MTestGetIntracommGeneral's communicators;
 * this library has COMM_WORLD only).  Every case runs with its operands in host memory
 * (`host`) or in device memory (`device`: hipMalloc, the path this library accelerates).
 *
 *   usage: mv2run -n N coll_suite {host|device} [case ...]
 *
 * Prints one line per case ("case errors seconds") on rank 0 and exits non-zero when any rank
 * counted an error.  The checks are the reference tests' own closed forms; file:line cites the
 * test each case restates. */
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static int g_dev, g_rank, g_size;

/* ---- operand buffers: host or device ------------------------------------------------- */
static void *ob_alloc(size_t bytes) {
    void *p = NULL;
    if (!bytes) bytes = 1;
    if (g_dev) {
        if (hipMalloc(&p, bytes) != hipSuccess) p = NULL;
    } else {
        p = malloc(bytes);
    }
    if (!p) {
        fprintf(stderr, "[%d] out of memory (%zu bytes)\n", g_rank, bytes);
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    return p;
}
static void ob_free(void *p) {
    if (g_dev) (void)hipFree(p);
    else free(p);
}
static void ob_put(void *ob, const void *h, size_t bytes) {  /* host values -> operand buffer */
    if (g_dev) (void)hipMemcpy(ob, h, bytes, hipMemcpyHostToDevice);
    else memcpy(ob, h, bytes);
}
static void ob_get(void *h, const void *ob, size_t bytes) {  /* operand buffer -> host copy */
    if (g_dev) (void)hipMemcpy(h, ob, bytes, hipMemcpyDeviceToHost);
    else memcpy(h, ob, bytes);
}
static void *xmalloc(size_t bytes) {
    void *p = malloc(bytes ? bytes : 1);
    if (!p) MPI_Abort(MPI_COMM_WORLD, 2);
    return p;
}
static int chk(int cond) { return cond ? 0 : 1; }

/* ---- user functions ----------------------------------------------------------------- */
/* allred3.c:29-62 / allred4.c:35-66: C = IN x INOUT per matrix (row-major, c(i,j) at j + i*m),
 * associative, not commutative */
static int g_mat;  /* matrix order of the current case */
static void op_matmul(void *in_, void *io_, int *len, MPI_Datatype *dt) {
    (void)dt;
    const int m = g_mat, mm = m * m;
    const int *in = (const int *)in_;
    int *io = (int *)io_;
    int col[256];
    for (int e = 0; e < *len; ++e, in += mm, io += mm)
        for (int j = 0; j < m; ++j) {
            for (int i = 0; i < m; ++i) {
                int s = 0;
                for (int k = 0; k < m; ++k) s += in[i * m + k] * io[k * m + j];
                col[i] = s;
            }
            for (int i = 0; i < m; ++i) io[i * m + j] = col[i];
        }
}
/* allred6.c:24-31: a sum declared non-commutative */
static void op_nc_isum(void *in_, void *io_, int *len, MPI_Datatype *dt) {
    (void)dt;
    const int *in = (const int *)in_;
    int *io = (int *)io_;
    for (int i = 0; i < *len; ++i) io[i] += in[i];
}
/* uoplong.c:26-38: triples of doubles -> (sum, max, min) */
static void op_triple(void *in_, void *io_, int *len, MPI_Datatype *dt) {
    (void)dt;
    const double *in = (const double *)in_;
    double *io = (double *)io_;
    for (int e = 0; e < *len; ++e, in += 3, io += 3) {
        io[0] += in[0];
        io[1] = io[1] > in[1] ? io[1] : in[1];
        io[2] = io[2] < in[2] ? io[2] : in[2];
    }
}
/* redscat2.c:22-56: left(x, y) = x, right(x, y) = y, both counting an operand that arrives out
 * of rank order (the operands are rank + i, so IN must never exceed INOUT); nc_sum = x + y */
static int g_order_err;
static void op_left(void *in_, void *io_, int *len, MPI_Datatype *dt) {
    (void)dt;
    const int *in = (const int *)in_;
    int *io = (int *)io_;
    for (int i = 0; i < *len; ++i) {
        g_order_err += in[i] > io[i];
        io[i] = in[i];
    }
}
static void op_right(void *in_, void *io_, int *len, MPI_Datatype *dt) {
    (void)dt;
    const int *in = (const int *)in_;
    const int *io = (const int *)io_;
    for (int i = 0; i < *len; ++i) g_order_err += in[i] > io[i];
}
static void op_nc_sum(void *in_, void *io_, int *len, MPI_Datatype *dt) {
    (void)dt;
    const int *in = (const int *)in_;
    int *io = (int *)io_;
    for (int i = 0; i < *len; ++i) io[i] = in[i] + io[i];
}

/* ---- cases -------------------------------------------------------------------------- */
/* allred2.c:30-48: in-place MPI_SUM over MPI_INT, counts 1 .. 32768 */
static int t_allred2(void) {
    int errs = 0;
    for (int count = 1; count < 65000; count *= 2) {
        int *h = xmalloc(count * sizeof(int));
        for (int i = 0; i < count; ++i) h[i] = g_rank + i;
        int *b = ob_alloc(count * sizeof(int));
        ob_put(b, h, count * sizeof(int));
        errs += MPI_Allreduce(MPI_IN_PLACE, b, count, MPI_INT, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
        ob_get(h, b, count * sizeof(int));
        for (int i = 0; i < count; ++i) errs += chk(h[i] == i * g_size + g_size * (g_size - 1) / 2);
        ob_free(b);
        free(h);
    }
    return errs;
}

/* allred3.c:70-112: rank r < n-1 holds the permutation exchanging r and r+1, rank n-1 the
 * right shift; their ordered product is the identity */
static void allred3_init(int *mat) {
    const int m = g_size;
    memset(mat, 0, sizeof(int) * m * m);
    if (g_rank < m - 1) {
        for (int i = 0; i < m; ++i) {
            int j = i;
            if (i == g_rank) j = (i + 1) % m;
            else if (i == (g_rank + 1) % m) j = (i + m - 1) % m;
            mat[i * m + j] = 1;
        }
    } else {
        for (int i = 0; i < m; ++i) mat[i * m + (i + 1) % m] = 1;
    }
}
static int t_allred3(void) {
    if (g_size < 2 || g_size > 256) return 0;
    const int m = g_size, bytes = m * m * (int)sizeof(int);
    g_mat = m;
    MPI_Op op;
    MPI_Datatype mt;
    MPI_Op_create(op_matmul, 0, &op);
    MPI_Type_contiguous(m * m, MPI_INT, &mt);
    MPI_Type_commit(&mt);
    int errs = 0, *h = xmalloc(bytes);
    int *a = ob_alloc(bytes), *b = ob_alloc(bytes);
    for (int pass = 0; pass < 2; ++pass) {  /* sendbuf -> recvbuf, then MPI_IN_PLACE */
        allred3_init(h);
        ob_put(pass ? b : a, h, bytes);
        errs += MPI_Allreduce(pass ? MPI_IN_PLACE : a, b, 1, mt, op, MPI_COMM_WORLD) != MPI_SUCCESS;
        ob_get(h, b, bytes);
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < m; ++j) errs += chk(h[i * m + j] == (i == j));
    }
    ob_free(a);
    ob_free(b);
    free(h);
    MPI_Type_free(&mt);
    MPI_Op_free(&op);
    return errs;
}

/* allred4.c:74-121, 199-228: 3x3 matrices I, A, B placed so that the ordered product is one
 * rotation; counts 1 .. n-1 matrices per rank */
static void allred4_init(int *mat) {
    int kind = 0;
    if (g_size == 2) kind = 1 + g_rank;
    else if (g_rank == g_size / 4) kind = 1;
    else if (g_rank == (3 * g_size) / 4) kind = 2;
    static const int ident[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    static const int mat_a[9] = {1, 0, 0, 0, 0, 1, 0, 1, 0};
    static const int mat_b[9] = {0, 1, 0, 1, 0, 0, 0, 0, 1};
    memcpy(mat, kind == 0 ? ident : kind == 1 ? mat_a : mat_b, sizeof(ident));
}
static int t_allred4(void) {
    static const int want[9] = {0, 1, 0, 0, 0, 1, 1, 0, 0};
    g_mat = 3;
    MPI_Op op;
    MPI_Datatype mt;
    MPI_Op_create(op_matmul, 0, &op);
    MPI_Type_contiguous(9, MPI_INT, &mt);
    MPI_Type_commit(&mt);
    int errs = 0;
    for (int count = 1; count < g_size; ++count) {
        const size_t bytes = (size_t)count * 9 * sizeof(int);
        int *h = xmalloc(bytes);
        int *a = ob_alloc(bytes), *b = ob_alloc(bytes);
        for (int pass = 0; pass < 2; ++pass) {
            for (int k = 0; k < count; ++k) allred4_init(h + 9 * k);
            ob_put(pass ? b : a, h, bytes);
            errs += MPI_Allreduce(pass ? MPI_IN_PLACE : a, b, count, mt, op, MPI_COMM_WORLD) != MPI_SUCCESS;
            ob_get(h, b, bytes);
            for (int k = 0; k < count * 9; ++k) errs += chk(h[k] == want[k % 9]);
        }
        ob_free(a);
        ob_free(b);
        free(h);
    }
    MPI_Type_free(&mt);
    MPI_Op_free(&op);
    return errs;
}

/* allred5.c:33-55: count = 2n, MPI_SUM of i */
static int t_allred5(void) {
    const int count = 2 * g_size;
    int *h = xmalloc(count * sizeof(int));
    int *a = ob_alloc(count * sizeof(int)), *b = ob_alloc(count * sizeof(int));
    for (int i = 0; i < count; ++i) h[i] = i;
    ob_put(a, h, count * sizeof(int));
    for (int i = 0; i < count; ++i) h[i] = -1;
    ob_put(b, h, count * sizeof(int));
    int errs = MPI_Allreduce(a, b, count, MPI_INT, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
    ob_get(h, b, count * sizeof(int));
    for (int i = 0; i < count; ++i) errs += chk(h[i] == i * g_size);
    ob_free(a);
    ob_free(b);
    free(h);
    return errs;
}

/* allred6.c:49-68: the non-commutative-declared sum, in place, counts 1 .. 32768 */
static int t_allred6(void) {
    MPI_Op op;
    MPI_Op_create(op_nc_isum, 0, &op);
    int errs = 0;
    for (int count = 1; count < 65000; count *= 2) {
        int *h = xmalloc(count * sizeof(int));
        for (int i = 0; i < count; ++i) h[i] = g_rank + i;
        int *b = ob_alloc(count * sizeof(int));
        ob_put(b, h, count * sizeof(int));
        errs += MPI_Allreduce(MPI_IN_PLACE, b, count, MPI_INT, op, MPI_COMM_WORLD) != MPI_SUCCESS;
        ob_get(h, b, count * sizeof(int));
        for (int i = 0; i < count; ++i) errs += chk(h[i] == i * g_size + g_size * (g_size - 1) / 2);
        ob_free(b);
        free(h);
    }
    MPI_Op_free(&op);
    return errs;
}

/* allredmany.c:22-25: 10000 back-to-back one-double MPI_SUM allreduces */
static int t_allredmany(void) {
    const double w = 10.0;
    double *a = ob_alloc(sizeof(double)), *b = ob_alloc(sizeof(double)), got = 0;
    ob_put(a, &w, sizeof w);
    int errs = 0;
    for (int i = 0; i < 10000; ++i) errs += MPI_Allreduce(a, b, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
    ob_get(&got, b, sizeof got);
    errs += chk(got == 10.0 * g_size);
    ob_free(a);
    ob_free(b);
    return errs;
}

/* uoplong.c:48-100: MPI_Reduce to 0 of MPI_Type_contiguous(3, MPI_DOUBLE) triples with the
 * (sum, max, min) user function, counts 1 .. 2^20 */
static int t_uoplong(void) {
    MPI_Op op;
    MPI_Datatype tt;
    MPI_Op_create(op_triple, 0, &op);
    MPI_Type_contiguous(3, MPI_DOUBLE, &tt);
    MPI_Type_commit(&tt);
    int errs = 0;
    for (int count = 1; count < 1200000; count += count) {
        const size_t bytes = (size_t)count * 3 * sizeof(double);
        double *h = xmalloc(bytes);
        double *a = ob_alloc(bytes), *b = ob_alloc(bytes);
        for (int i = 0; i < 3 * count; ++i) h[i] = 1 + (i & 3);
        ob_put(a, h, bytes);
        for (int i = 0; i < 3 * count; ++i) h[i] = -1;
        ob_put(b, h, bytes);
        errs += MPI_Reduce(a, b, count, tt, op, 0, MPI_COMM_WORLD) != MPI_SUCCESS;
        if (g_rank == 0) {
            ob_get(h, b, bytes);
            for (int i = 0; i < 3 * count; i += 3) {
                errs += chk(h[i] == (double)g_size * (1 + (i & 3)));
                errs += chk(h[i + 1] == 1 + ((i + 1) & 3));
                errs += chk(h[i + 2] == 1 + ((i + 2) & 3));
            }
        }
        ob_free(a);
        ob_free(b);
        free(h);
    }
    MPI_Type_free(&tt);
    MPI_Op_free(&op);
    return errs;
}

/* redscat2.c:78-125 / red_scat_block2.c: non-commutative left / right / nc_sum, block sizes
 * 1 .. 128, MPI_Reduce_scatter (blk = 0) or MPI_Reduce_scatter_block (blk = 1) */
static int redscat_noncomm(int blk) {
    MPI_Op ops[3];
    MPI_Op_create(op_left, 0, &ops[0]);
    MPI_Op_create(op_right, 0, &ops[1]);
    MPI_Op_create(op_nc_sum, 0, &ops[2]);
    int errs = 0;
    g_order_err = 0;
    int *counts = xmalloc(g_size * sizeof(int));
    for (int bs = 1; bs < 256; bs *= 2) {
        const size_t sbytes = (size_t)bs * g_size * sizeof(int), rbytes = (size_t)bs * sizeof(int);
        int *h = xmalloc(sbytes);
        int *s = ob_alloc(sbytes), *r = ob_alloc(rbytes);
        for (int i = 0; i < bs * g_size; ++i) h[i] = g_rank + i;
        ob_put(s, h, sbytes);
        for (int i = 0; i < g_size; ++i) counts[i] = bs;
        for (int k = 0; k < 3; ++k) {
            for (int i = 0; i < bs; ++i) h[i] = (int)0xdeadbeef;
            ob_put(r, h, rbytes);
            const int rc = blk ? MPI_Reduce_scatter_block(s, r, bs, MPI_INT, ops[k], MPI_COMM_WORLD)
                               : MPI_Reduce_scatter(s, r, counts, MPI_INT, ops[k], MPI_COMM_WORLD);
            errs += rc != MPI_SUCCESS;
            ob_get(h, r, rbytes);
            for (int i = 0; i < bs; ++i) {
                const int x = g_rank * bs + i;
                const int want = k == 0 ? x : k == 1 ? (g_size - 1) + x : g_size * x + (g_size - 1) * g_size / 2;
                errs += chk(h[i] == want);
            }
        }
        ob_free(s);
        ob_free(r);
        free(h);
    }
    free(counts);
    for (int k = 0; k < 3; ++k) MPI_Op_free(&ops[k]);
    return errs + g_order_err;
}
static int t_redscat2(void) { return redscat_noncomm(0); }
static int t_red_scat_block2(void) { return redscat_noncomm(1); }

/* redscat3.c:43-99 / redscatblk3.c:34-77: 1 Mi ints split over the ranks, MPI_SUM, then the
 * same in place */
static int redscat_big(int blk) {
    const int my = (1024 * 1024) / g_size;
    const size_t sbytes = (size_t)my * g_size * sizeof(int), rbytes = (size_t)my * sizeof(int);
    int *counts = xmalloc(g_size * sizeof(int));
    for (int i = 0; i < g_size; ++i) counts[i] = my;
    int *h = xmalloc(sbytes);
    for (int i = 0; i < g_size; ++i)
        for (int j = 0; j < my; ++j) h[(size_t)i * my + j] = g_rank + i;
    int *s = ob_alloc(sbytes), *r = ob_alloc(rbytes);
    ob_put(s, h, sbytes);
    for (int i = 0; i < my; ++i) h[i] = -1;
    ob_put(r, h, rbytes);
    const int want = g_size * g_rank + (g_size - 1) * g_size / 2;
    int errs = (blk ? MPI_Reduce_scatter_block(s, r, my, MPI_INT, MPI_SUM, MPI_COMM_WORLD)
                    : MPI_Reduce_scatter(s, r, counts, MPI_INT, MPI_SUM, MPI_COMM_WORLD)) != MPI_SUCCESS;
    ob_get(h, r, rbytes);
    for (int i = 0; i < my; ++i) errs += chk(h[i] == want);
    errs += (blk ? MPI_Reduce_scatter_block(MPI_IN_PLACE, s, my, MPI_INT, MPI_SUM, MPI_COMM_WORLD)
                 : MPI_Reduce_scatter(MPI_IN_PLACE, s, counts, MPI_INT, MPI_SUM, MPI_COMM_WORLD)) != MPI_SUCCESS;
    ob_get(h, s, rbytes);
    for (int i = 0; i < my; ++i) errs += chk(h[i] == want);
    ob_free(s);
    ob_free(r);
    free(h);
    free(counts);
    return errs;
}
static int t_redscat3(void) { return redscat_big(0); }
static int t_redscatblk3(void) { return redscat_big(1); }

/* reduce.c:33-52: MPI_SUM of i to every root, counts 1 .. 65536 */
static int t_reduce(void) {
    int errs = 0;
    for (int count = 1; count < 130000; count *= 2) {
        int *h = xmalloc(count * sizeof(int));
        int *s = ob_alloc(count * sizeof(int)), *r = ob_alloc(count * sizeof(int));
        for (int root = 0; root < g_size; ++root) {
            for (int i = 0; i < count; ++i) h[i] = i;
            ob_put(s, h, count * sizeof(int));
            for (int i = 0; i < count; ++i) h[i] = -1;
            ob_put(r, h, count * sizeof(int));
            errs += MPI_Reduce(s, r, count, MPI_INT, MPI_SUM, root, MPI_COMM_WORLD) != MPI_SUCCESS;
            if (g_rank == root) {
                ob_get(h, r, count * sizeof(int));
                for (int i = 0; i < count; ++i) errs += chk(h[i] == i * g_size);
            }
        }
        ob_free(s);
        ob_free(r);
        free(h);
    }
    return errs;
}

/* allgather2.c:29-45: in place (sendcount -1, MPI_DATATYPE_NULL), doubles, counts 1 .. 8192 */
static int t_allgather2(void) {
    int errs = 0;
    for (int count = 1; count < 9000; count *= 2) {
        const size_t bytes = (size_t)count * g_size * sizeof(double);
        double *h = xmalloc(bytes);
        for (int i = 0; i < count * g_size; ++i) h[i] = -1;
        for (int i = 0; i < count; ++i) h[g_rank * count + i] = g_rank * count + i;
        double *v = ob_alloc(bytes);
        ob_put(v, h, bytes);
        errs += MPI_Allgather(MPI_IN_PLACE, -1, MPI_DATATYPE_NULL, v, count, MPI_DOUBLE, MPI_COMM_WORLD) != MPI_SUCCESS;
        ob_get(h, v, bytes);
        for (int i = 0; i < count * g_size; ++i) errs += chk(h[i] == i);
        ob_free(v);
        free(h);
    }
    return errs;
}

/* allgather3.c:29-56: doubles, counts 1 .. 8192; then a zero-byte in-place gather into NULL */
static int t_allgather3(void) {
    int errs = 0;
    for (int count = 1; count < 9000; count *= 2) {
        const size_t bytes = (size_t)count * g_size * sizeof(double);
        double *h = xmalloc(bytes);
        for (int i = 0; i < count; ++i) h[i] = g_rank * count + i;
        double *in = ob_alloc(count * sizeof(double)), *out = ob_alloc(bytes);
        ob_put(in, h, count * sizeof(double));
        errs += MPI_Allgather(in, count, MPI_DOUBLE, out, count, MPI_DOUBLE, MPI_COMM_WORLD) != MPI_SUCCESS;
        ob_get(h, out, bytes);
        for (int i = 0; i < count * g_size; ++i) errs += chk(h[i] == i);
        ob_free(in);
        ob_free(out);
        free(h);
    }
    errs += MPI_Allgather(MPI_IN_PLACE, -1, MPI_DATATYPE_NULL, NULL, 0, MPI_BYTE, MPI_COMM_WORLD) != MPI_SUCCESS;
    return errs;
}

/* bcasttest.c:18-67: MPI_INT broadcasts of 100, 64 Ki, 128 Ki and 1 Mi elements from rank 0,
 * five repetitions each, every repetition with new values */
static int t_bcasttest(void) {
    static const int sizes[4] = {100, 64 * 1024, 128 * 1024, 1024 * 1024};
    int errs = 0;
    int *h = xmalloc(sizes[3] * sizeof(int));
    int *b = ob_alloc(sizes[3] * sizeof(int));
    for (int n = 0; n < 4; ++n)
        for (int rep = 0; rep < 5; ++rep) {
            const int tag = n * 5 + rep;
            for (int i = 0; i < sizes[n]; ++i) h[i] = g_rank == 0 ? 1000000 * tag + i : -1 - tag;
            ob_put(b, h, sizes[n] * sizeof(int));
            errs += MPI_Bcast(b, sizes[n], MPI_INT, 0, MPI_COMM_WORLD) != MPI_SUCCESS;
            ob_get(h, b, sizes[n] * sizeof(int));
            for (int i = 0; i < sizes[n]; ++i) errs += chk(h[i] == 1000000 * tag + i);
        }
    ob_free(b);
    free(h);
    return errs;
}

/* bcastzerotype.c:28-48: a broadcast of a zero-size type leaves every buffer as it was */
static int t_bcastzerotype(void) {
    MPI_Datatype zt;
    int sz = -1, errs = 0, h[10];
    MPI_Type_contiguous(0, MPI_INT, &zt);
    MPI_Type_commit(&zt);
    MPI_Type_size(zt, &sz);
    errs += chk(sz == 0);
    for (int i = 0; i < 10; ++i) h[i] = g_rank * 10 + i;
    int *b = ob_alloc(sizeof h);
    ob_put(b, h, sizeof h);
    errs += MPI_Bcast(b, 10, zt, 0, MPI_COMM_WORLD) != MPI_SUCCESS;
    ob_get(h, b, sizeof h);
    for (int i = 0; i < 10; ++i) errs += chk(h[i] == g_rank * 10 + i);
    ob_free(b);
    MPI_Type_free(&zt);
    return errs;
}

/* op_commutative.c:59-101: every predefined op is commutative; a user op is what it declared */
static int t_op_commutative(void) {
    static const MPI_Op pre[] = {MPI_MAX, MPI_MIN, MPI_SUM, MPI_PROD, MPI_LAND, MPI_BAND,
                                 MPI_LOR, MPI_BOR, MPI_LXOR, MPI_BXOR, MPI_MAXLOC, MPI_MINLOC};
    int errs = 0, c = 0;
    for (size_t k = 0; k < sizeof pre / sizeof pre[0]; ++k) {
        MPI_Op_commutative(pre[k], &c);
        errs += chk(c == 1);
    }
    MPI_Op cu, nu;
    MPI_Op_create(op_nc_isum, 1, &cu);
    MPI_Op_create(op_nc_isum, 0, &nu);
    MPI_Op_commutative(cu, &c);
    errs += chk(c == 1);
    MPI_Op_commutative(nu, &c);
    errs += chk(c == 0);
    MPI_Op_free(&nu);
    MPI_Op_free(&cu);
    return errs;
}

/* red3.c / red4.c: MPI_Reduce of permutation matrices with the matrix product, every root,
 * then in place at the root with NULL receive buffers elsewhere.  red3: rank r < n-1 exchanges
 * r and r+1, the last rank holds the identity; red4: every rank exchanges r and (r+1) % n.  The
 * expected answer is the ordered product P_0 ... P_{n-1}, computed here with the same function
 * (red4.c:16-20: independent of the root). */
static void swap_perm(int m, int r, int *mat) {
    memset(mat, 0, sizeof(int) * m * m);
    for (int i = 0; i < m; ++i) {
        int j = i;
        if (i == r) j = (i + 1) % m;
        else if (i == (r + 1) % m) j = (i + m - 1) % m;
        mat[i * m + j] = 1;
    }
}
static void red_mat(int red4, int r, int *mat) {
    const int m = g_size;
    if (!red4 && r == m - 1) {
        memset(mat, 0, sizeof(int) * m * m);
        for (int i = 0; i < m; ++i) mat[i * m + i] = 1;
    } else {
        swap_perm(m, r, mat);
    }
}
static int red_noncomm(int red4) {
    if (g_size < 2 || g_size > 256) return 0;
    const int m = g_size, bytes = m * m * (int)sizeof(int);
    g_mat = m;
    MPI_Op op;
    MPI_Datatype mt;
    MPI_Op_create(op_matmul, 0, &op);
    MPI_Type_contiguous(m * m, MPI_INT, &mt);
    MPI_Type_commit(&mt);
    int *want = xmalloc(bytes), *tmp = xmalloc(bytes), *h = xmalloc(bytes), one = 1;
    red_mat(red4, m - 1, want);
    for (int r = m - 2; r >= 0; --r) {  /* want = P_r x want */
        red_mat(red4, r, tmp);
        op_matmul(tmp, want, &one, &mt);
    }
    int errs = 0;
    int *a = ob_alloc(bytes), *b = ob_alloc(bytes);
    for (int root = 0; root < m; ++root)
        for (int pass = 0; pass < 2; ++pass) {
            red_mat(red4, g_rank, h);
            ob_put(pass ? b : a, h, bytes);
            const void *s = pass && g_rank == root ? MPI_IN_PLACE : pass ? (const void *)b : (const void *)a;
            void *r = pass && g_rank != root ? NULL : b;
            errs += MPI_Reduce(s, r, 1, mt, op, root, MPI_COMM_WORLD) != MPI_SUCCESS;
            if (g_rank == root) {
                ob_get(h, b, bytes);
                errs += chk(memcmp(h, want, bytes) == 0);
            }
        }
    ob_free(a);
    ob_free(b);
    free(want);
    free(tmp);
    free(h);
    MPI_Type_free(&mt);
    MPI_Op_free(&op);
    return errs;
}
static int t_red3(void) { return red_noncomm(0); }
static int t_red4(void) { return red_noncomm(1); }

/* longuser.c:16-60: a commutative user sum of doubles (+1 on odd ranks, -1 on even), counts
 * 1 .. 65536 */
static void op_dsum(void *in_, void *io_, int *len, MPI_Datatype *dt) {
    (void)dt;
    const double *in = (const double *)in_;
    double *io = (double *)io_;
    for (int i = 0; i < *len; ++i) io[i] = in[i] + io[i];
}
static int t_longuser(void) {
    MPI_Op op;
    MPI_Op_create(op_dsum, 1, &op);
    int errs = 0;
    const double want = (g_size & 1) ? -1.0 : 0.0;
    for (int count = 1; count < 100000; count *= 2) {
        double *h = xmalloc(count * sizeof(double));
        double *a = ob_alloc(count * sizeof(double)), *b = ob_alloc(count * sizeof(double));
        for (int i = 0; i < count; ++i) h[i] = (g_rank & 1) ? 1.0 : -1.0;
        ob_put(a, h, count * sizeof(double));
        for (int i = 0; i < count; ++i) h[i] = 100.0;
        ob_put(b, h, count * sizeof(double));
        errs += MPI_Allreduce(a, b, count, MPI_DOUBLE, op, MPI_COMM_WORLD) != MPI_SUCCESS;
        ob_get(h, b, count * sizeof(double));
        for (int i = 0; i < count; ++i) errs += chk(h[i] == want);
        ob_free(a);
        ob_free(b);
        free(h);
    }
    MPI_Op_free(&op);
    return errs;
}

/* one int operand / result in operand memory */
static int reduce_int(int v, MPI_Op op, int root, int *out) {
    int *a = ob_alloc(sizeof(int)), *b = ob_alloc(sizeof(int)), init = -100;
    ob_put(a, &v, sizeof v);
    ob_put(b, &init, sizeof init);
    int errs = MPI_Reduce(a, b, 1, MPI_INT, op, root, MPI_COMM_WORLD) != MPI_SUCCESS;
    errs += MPI_Bcast(b, 1, MPI_INT, root, MPI_COMM_WORLD) != MPI_SUCCESS;
    ob_get(out, b, sizeof(int));
    ob_free(a);
    ob_free(b);
    return errs;
}

/* coll8.c: MPI_Reduce of the rank with SUM, MIN, MAX to rank 0 */
static int t_coll8(void) {
    int errs = 0, r = 0;
    errs += reduce_int(g_rank, MPI_SUM, 0, &r) + chk(r == g_size * (g_size - 1) / 2);
    errs += reduce_int(g_rank, MPI_MIN, 0, &r) + chk(r == 0);
    errs += reduce_int(g_rank, MPI_MAX, 0, &r) + chk(r == g_size - 1);
    return errs;
}

/* coll9.c: a commutative user sum, MPI_Reduce to rank 0 */
static int t_coll9(void) {
    MPI_Op op;
    MPI_Op_create(op_nc_isum, 1, &op);
    int r = 0, errs = reduce_int(g_rank, op, 0, &r) + chk(r == g_size * (g_size - 1) / 2);
    MPI_Op_free(&op);
    return errs;
}

/* coll10.c:19-35: IN must always come from lower ranks than INOUT (the computation is in rank
 * order, independent of the root); a violation yields 100000.  Reduce to rank n-1. */
static void op_assoc(void *in_, void *io_, int *len, MPI_Datatype *dt) {
    (void)dt;
    const int *in = (const int *)in_;
    int *io = (int *)io_;
    for (int i = 0; i < *len; ++i) io[i] = io[i] <= in[i] ? 100000 : in[i];
}
static int t_coll10(void) {
    MPI_Op op;
    MPI_Op_create(op_assoc, 0, &op);
    int r = 0, errs = reduce_int(g_rank, op, g_size - 1, &r) + chk(r == 0);
    MPI_Op_free(&op);
    return errs;
}

/* coll12.c: MAXLOC (Reduce + Bcast) and MINLOC (Allreduce) of MPI_DOUBLE_INT over a 2-entry
 * table: entry i is rank + 1 (negated for MINLOC) from rank i on, 0 below; entry i's location
 * is rank i */
struct di {
    double v;
    int loc;
};
static int t_coll12(void) {
    struct di in[2], out[2];
    int errs = 0;
    struct di *a = ob_alloc(sizeof in), *b = ob_alloc(sizeof out);
    for (int pass = 0; pass < 2; ++pass) {
        memset(in, 0, sizeof in);
        for (int i = 0; i < 2; ++i) {
            in[i].v = i >= g_rank ? (pass ? -1.0 : 1.0) * (g_rank + 1.0) : 0.0;
            in[i].loc = g_rank;
        }
        ob_put(a, in, sizeof in);
        if (!pass) {
            errs += MPI_Reduce(a, b, 2, MPI_DOUBLE_INT, MPI_MAXLOC, 0, MPI_COMM_WORLD) != MPI_SUCCESS;
            errs += MPI_Bcast(b, 2, MPI_DOUBLE_INT, 0, MPI_COMM_WORLD) != MPI_SUCCESS;
        } else {
            errs += MPI_Allreduce(a, b, 2, MPI_DOUBLE_INT, MPI_MINLOC, MPI_COMM_WORLD) != MPI_SUCCESS;
        }
        ob_get(out, b, sizeof out);
        for (int i = 0; i < 2; ++i)
            if (i % g_size == g_rank) errs += chk(out[i].loc == g_rank);
    }
    ob_free(a);
    ob_free(b);
    return errs;
}

/* iallred.c: an MPI_Iallreduce left in flight across a blocking MPI_Allreduce */
static int t_iallred(void) {
    const int one = 1, two = 2;
    int *a = ob_alloc(sizeof(int)), *b = ob_alloc(sizeof(int)), *c = ob_alloc(sizeof(int)), *d = ob_alloc(sizeof(int));
    ob_put(a, &one, sizeof one);
    ob_put(c, &two, sizeof two);
    MPI_Request req;
    int errs = MPI_Iallreduce(a, b, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD, &req) != MPI_SUCCESS;
    errs += MPI_Allreduce(c, d, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
    errs += MPI_Wait(&req, MPI_STATUS_IGNORE) != MPI_SUCCESS;
    int isum = 0, sum = 0;
    ob_get(&isum, b, sizeof isum);
    ob_get(&sum, d, sizeof sum);
    errs += chk(isum == g_size && sum == 2 * g_size);
    ob_free(a);
    ob_free(b);
    ob_free(c);
    ob_free(d);
    return errs;
}

/* nonblocking2.c (the collectives this library provides): Ibcast of 10 ints and of 17 signed
 * chars (bytes past them untouched), Ibarrier, Ireduce with MPI_SUM and with a user op freed
 * before the wait, Iallreduce, Ireduce_scatter and Ireduce_scatter_block (the receive buffer
 * past the rank's block untouched), Iallgather; COUNT = 10 */
static int t_nonblocking2(void) {
    enum { CNT = 10, PRIME = 17 };
    const int n = g_size, nb = CNT * n * (int)sizeof(int);
    int *h = xmalloc(nb), *g = xmalloc(nb), *counts = xmalloc(n * sizeof(int));
    int *buf = ob_alloc(nb), *rbuf = ob_alloc(nb);
    MPI_Request req;
    int errs = 0;
    const int tri = n * (n - 1) / 2;
    /* Ibcast of COUNT ints */
    for (int i = 0; i < CNT; ++i) h[i] = g_rank == 0 ? i : -1;
    ob_put(buf, h, CNT * sizeof(int));
    errs += MPI_Ibcast(buf, CNT, MPI_INT, 0, MPI_COMM_WORLD, &req) != MPI_SUCCESS;
    errs += MPI_Wait(&req, MPI_STATUS_IGNORE) != MPI_SUCCESS;
    ob_get(h, buf, CNT * sizeof(int));
    for (int i = 0; i < CNT; ++i) errs += chk(h[i] == i);
    /* Ibcast of PRIME signed chars inside a larger buffer */
    signed char *hc = (signed char *)h;
    for (int i = 0; i < nb; ++i) hc[i] = i < PRIME ? (g_rank == 0 ? (signed char)i : (signed char)0xdb) : (signed char)0xbf;
    ob_put(buf, h, nb);
    errs += MPI_Ibcast(buf, PRIME, MPI_SIGNED_CHAR, 0, MPI_COMM_WORLD, &req) != MPI_SUCCESS;
    errs += MPI_Wait(&req, MPI_STATUS_IGNORE) != MPI_SUCCESS;
    ob_get(h, buf, nb);
    for (int i = 0; i < nb; ++i) errs += chk(hc[i] == (i < PRIME ? (signed char)i : (signed char)0xbf));
    /* Ibarrier */
    errs += MPI_Ibarrier(MPI_COMM_WORLD, &req) != MPI_SUCCESS;
    errs += MPI_Wait(&req, MPI_STATUS_IGNORE) != MPI_SUCCESS;
    /* Ireduce (SUM, then a user sum freed before the wait) and Iallreduce */
    for (int k = 0; k < 3; ++k) {
        for (int i = 0; i < CNT; ++i) {
            h[i] = g_rank + i;
            g[i] = (int)0xdeadbeef;
        }
        ob_put(buf, h, CNT * sizeof(int));
        ob_put(rbuf, g, CNT * sizeof(int));
        MPI_Op op = MPI_SUM;
        if (k == 1) MPI_Op_create(op_nc_isum, 1, &op);
        if (k < 2) errs += MPI_Ireduce(buf, rbuf, CNT, MPI_INT, op, 0, MPI_COMM_WORLD, &req) != MPI_SUCCESS;
        else errs += MPI_Iallreduce(buf, rbuf, CNT, MPI_INT, op, MPI_COMM_WORLD, &req) != MPI_SUCCESS;
        if (k == 1) MPI_Op_free(&op);
        errs += MPI_Wait(&req, MPI_STATUS_IGNORE) != MPI_SUCCESS;
        if (k == 2 || g_rank == 0) {
            ob_get(g, rbuf, CNT * sizeof(int));
            for (int i = 0; i < CNT; ++i) errs += chk(g[i] == tri + i * n);
        }
    }
    /* Ireduce_scatter / Ireduce_scatter_block: block i of every rank holds rank + i */
    for (int blk = 0; blk < 2; ++blk) {
        for (int i = 0; i < n; ++i) {
            counts[i] = CNT;
            for (int j = 0; j < CNT; ++j) {
                h[i * CNT + j] = g_rank + i;
                g[i * CNT + j] = (int)0xdeadbeef;
            }
        }
        ob_put(buf, h, nb);
        ob_put(rbuf, g, nb);
        if (blk) errs += MPI_Ireduce_scatter_block(buf, rbuf, CNT, MPI_INT, MPI_SUM, MPI_COMM_WORLD, &req) != MPI_SUCCESS;
        else errs += MPI_Ireduce_scatter(buf, rbuf, counts, MPI_INT, MPI_SUM, MPI_COMM_WORLD, &req) != MPI_SUCCESS;
        errs += MPI_Wait(&req, MPI_STATUS_IGNORE) != MPI_SUCCESS;
        ob_get(g, rbuf, nb);
        for (int j = 0; j < CNT; ++j) errs += chk(g[j] == n * g_rank + tri);
        for (int j = CNT; j < CNT * n; ++j) errs += chk(g[j] == (int)0xdeadbeef);
    }
    /* Iallgather */
    for (int i = 0; i < n * CNT; ++i) {
        h[i] = g_rank + i;
        g[i] = (int)0xdeadbeef;
    }
    ob_put(buf, h, nb);
    ob_put(rbuf, g, nb);
    errs += MPI_Iallgather(buf, CNT, MPI_INT, rbuf, CNT, MPI_INT, MPI_COMM_WORLD, &req) != MPI_SUCCESS;
    errs += MPI_Wait(&req, MPI_STATUS_IGNORE) != MPI_SUCCESS;
    ob_get(g, rbuf, nb);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < CNT; ++j) errs += chk(g[i * CNT + j] == i + j);
    ob_free(buf);
    ob_free(rbuf);
    free(h);
    free(g);
    free(counts);
    return errs;
}

static const struct {
    const char *name;
    int (*fn)(void);
} kCases[] = {
    {"allred2", t_allred2},         {"allred3", t_allred3},
    {"allred4", t_allred4},         {"allred5", t_allred5},
    {"allred6", t_allred6},         {"allredmany", t_allredmany},
    {"uoplong", t_uoplong},         {"redscat2", t_redscat2},
    {"red_scat_block2", t_red_scat_block2}, {"redscat3", t_redscat3},
    {"redscatblk3", t_redscatblk3}, {"reduce", t_reduce},
    {"allgather2", t_allgather2},   {"allgather3", t_allgather3},
    {"bcasttest", t_bcasttest},     {"bcastzerotype", t_bcastzerotype},
    {"op_commutative", t_op_commutative},
    {"red3", t_red3},               {"red4", t_red4},
    {"longuser", t_longuser},       {"coll8", t_coll8},
    {"coll9", t_coll9},             {"coll10", t_coll10},
    {"coll12", t_coll12},           {"iallred", t_iallred},
    {"nonblocking2", t_nonblocking2},
};

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
    if (argc < 2 || (strcmp(argv[1], "host") && strcmp(argv[1], "device"))) {
        fprintf(stderr, "usage: coll_suite {host|device} [case ...]\n");
        return 2;
    }
    g_dev = !strcmp(argv[1], "device");
    MPI_Init(&argc, &argv);
    MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN);
    MPI_Comm_rank(MPI_COMM_WORLD, &g_rank);
    MPI_Comm_size(MPI_COMM_WORLD, &g_size);
    int total = 0, ran = 0;
    for (size_t k = 0; k < sizeof kCases / sizeof kCases[0]; ++k) {
        int wanted = argc <= 2;
        for (int a = 2; a < argc; ++a) wanted |= !strcmp(argv[a], kCases[k].name);
        if (!wanted) continue;
        const double t0 = now_s();
        int errs = kCases[k].fn(), all = 0;
        MPI_Allreduce(&errs, &all, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
        if (g_rank == 0) {
            printf("%s %s %d %.3f\n", argv[1], kCases[k].name, all, now_s() - t0);
            fflush(stdout);
        }
        total += all;
        ++ran;
    }
    if (g_rank == 0) printf("%s TOTAL %d cases %d\n", argv[1], total, ran);
    MPI_Finalize();
    return total ? 1 : 0;
}
