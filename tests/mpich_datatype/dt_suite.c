/* dt_suite.c — the reference's MPI_Pack / MPI_Unpack tests (MPICH test/mpi/datatype, shipped
 * with MVAPICH2 2.3.7) restated as one self-checking C program over the drop-in libmpi.so:
 * the same type constructors, buffer contents and expected layouts as each test program.
 * Operands live in host memory (`host`) or device memory (`device`: hipMalloc — the device
 * pack kernels); the pack buffer lives on the same side.
 *
 *   usage: dt_suite {host|device} [case ...]
 *
 * Prints "mode case errors" per case and exits non-zero when any case counted an error.
 * file:line cites the test each case restates. */
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int g_dev;

static void *ob_alloc(size_t bytes) {
    void *p = NULL;
    if (!bytes) bytes = 1;
    if (g_dev) {
        if (hipMalloc(&p, bytes) != hipSuccess) p = NULL;
    } else {
        p = malloc(bytes);
    }
    if (!p) MPI_Abort(MPI_COMM_WORLD, 2);
    return p;
}
static void ob_free(void *p) {
    if (g_dev) (void)hipFree(p);
    else free(p);
}
static void ob_put(void *ob, const void *h, size_t bytes) {
    if (g_dev) (void)hipMemcpy(ob, h, bytes, hipMemcpyHostToDevice);
    else memcpy(ob, h, bytes);
}
static void ob_get(void *h, const void *ob, size_t bytes) {
    if (g_dev) (void)hipMemcpy(h, ob, bytes, hipMemcpyDeviceToHost);
    else memcpy(h, ob, bytes);
}
static int chk(int cond) { return cond ? 0 : 1; }

/* Pack `count` x `t` from host image `src` (bytes of the operand's span) into a pack buffer,
 * clear the operand to `fill`, unpack back; `img` receives the operand afterwards.  Returns
 * the MPI error count; *packed (if given) receives the packed bytes (host copy). */
static int pack_roundtrip(const void *src, size_t span, int count, MPI_Datatype t, int fill, void *img,
                          void *packed, int *packed_size) {
    int psize = 0, pos = 0, errs = 0;
    MPI_Pack_size(count, t, MPI_COMM_WORLD, &psize);
    void *ob = ob_alloc(span), *pb = ob_alloc((size_t)psize);
    ob_put(ob, src, span);
    errs += MPI_Pack(ob, count, t, pb, psize, &pos, MPI_COMM_WORLD) != MPI_SUCCESS;
    if (packed) ob_get(packed, pb, (size_t)pos);
    if (packed_size) *packed_size = pos;
    const int used = pos;
    unsigned char *blank = malloc(span ? span : 1);
    memset(blank, fill, span);
    ob_put(ob, blank, span);
    free(blank);
    pos = 0;
    errs += MPI_Unpack(pb, used, &pos, ob, count, t, MPI_COMM_WORLD) != MPI_SUCCESS;
    errs += chk(pos == used);
    ob_get(img, ob, span);
    ob_free(ob);
    ob_free(pb);
    return errs;
}

/* simple-pack.c:95-170: vector(2,1,2) of vector(2,1,2,INT) over a 3x3 int array: the type map
 * is elements 0, 2, 6, 8; size 4 ints */
static int t_simple_pack_nested(void) {
    MPI_Datatype in, out;
    MPI_Type_vector(2, 1, 2, MPI_INT, &in);
    MPI_Type_vector(2, 1, 2, in, &out);
    MPI_Type_commit(&out);
    int sz = 0, errs = 0;
    MPI_Type_size(out, &sz);
    errs += chk(sz == 4 * (int)sizeof(int));
    const int arr[9] = {1, -1, 2, -2, -3, -4, 3, -5, 4};
    int img[9], pk[4], psz = 0;
    errs += pack_roundtrip(arr, sizeof arr, 1, out, 0, img, pk, &psz);
    errs += chk(psz == sz);
    for (int k = 0; k < 4; ++k) errs += chk(pk[k] == k + 1);
    for (int i = 0; i < 9; ++i) errs += chk(img[i] == (i == 0 ? 1 : i == 2 ? 2 : i == 6 ? 3 : i == 8 ? 4 : 0));
    MPI_Type_free(&out);
    MPI_Type_free(&in);
    return errs;
}

/* simple-pack.c:180-250: vector(10, 2, 2, INT) is 20 contiguous ints */
static int t_simple_pack_contig_vector(void) {
    MPI_Datatype t;
    MPI_Type_vector(10, 2, 2, MPI_INT, &t);
    MPI_Type_commit(&t);
    int arr[20], img[20], pk[20], psz = 0, sz = 0, errs = 0;
    for (int i = 0; i < 20; ++i) arr[i] = i;
    MPI_Type_size(t, &sz);
    errs += chk(sz == 20 * (int)sizeof(int));
    errs += pack_roundtrip(arr, sizeof arr, 1, t, 0, img, pk, &psz);
    errs += chk(psz == sz);
    for (int i = 0; i < 20; ++i) errs += chk(pk[i] == i && img[i] == i);
    MPI_Type_free(&t);
    return errs;
}

/* transpose-pack.c:40-80: hvector(100, 1, sizeof(int)) of a 100-int column packs a 100x100
 * matrix transposed; unpacked as 10000 MPI_INT it is the transpose */
static int t_transpose_pack(void) {
    MPI_Datatype row, xpose;
    MPI_Type_vector(100, 1, 100, MPI_INT, &row);
    MPI_Type_create_hvector(100, 1, sizeof(int), row, &xpose);
    MPI_Type_commit(&xpose);
    static int a[100][100], b[100][100];
    for (int i = 0; i < 100; ++i)
        for (int j = 0; j < 100; ++j) a[i][j] = i * 1000 + j;
    int psize = 0, pos = 0, errs = 0;
    MPI_Pack_size(1, xpose, MPI_COMM_WORLD, &psize);
    void *oa = ob_alloc(sizeof a), *ob = ob_alloc(sizeof b), *pb = ob_alloc(psize);
    ob_put(oa, a, sizeof a);
    errs += MPI_Pack(oa, 1, xpose, pb, psize, &pos, MPI_COMM_WORLD) != MPI_SUCCESS;
    pos = 0;
    errs += MPI_Unpack(pb, psize, &pos, ob, 100 * 100, MPI_INT, MPI_COMM_WORLD) != MPI_SUCCESS;
    ob_get(b, ob, sizeof b);
    for (int i = 0; i < 100; ++i)
        for (int j = 0; j < 100; ++j) errs += chk(b[i][j] == a[j][i]);
    ob_free(oa);
    ob_free(ob);
    ob_free(pb);
    MPI_Type_free(&xpose);
    MPI_Type_free(&row);
    return errs;
}

/* triangular-pack.c:35-80: indexed blocks i+1 at 100 i select the lower triangle; unpacking
 * into a zeroed matrix fills it and leaves the upper triangle zero */
static int t_triangular_pack(void) {
    int blk[100], disp[100];
    for (int i = 0; i < 100; ++i) {
        blk[i] = i + 1;
        disp[i] = 100 * i;
    }
    MPI_Datatype lt;
    MPI_Type_indexed(100, blk, disp, MPI_INT, &lt);
    MPI_Type_commit(&lt);
    static int a[100][100], b[100][100];
    for (int i = 0; i < 100; ++i)
        for (int j = 0; j < 100; ++j) a[i][j] = 1000 * i + j;
    int errs = pack_roundtrip(a, sizeof a, 1, lt, 0, b, NULL, NULL);
    for (int i = 0; i < 100; ++i)
        for (int j = 0; j < 100; ++j) errs += chk(b[i][j] == (j > i ? 0 : 1000 * i + j));
    MPI_Type_free(&lt);
    return errs;
}

/* slice-pack.c:35-90: a 9x9x9 slice of a 100^3 int array (every other element of a row,
 * rows 2.., planes 0..) packed from &a[0][2][1] and unpacked contiguously */
static int t_slice_pack(void) {
    MPI_Datatype one, two, three;
    MPI_Type_vector(9, 1, 2, MPI_INT, &one);
    MPI_Type_create_hvector(9, 1, 100 * sizeof(int), one, &two);
    MPI_Type_create_hvector(9, 1, 100 * 100 * sizeof(int), two, &three);
    MPI_Type_commit(&three);
    const size_t n = 100 * 100 * 100;
    int *a = malloc(n * sizeof(int)), e[9][9][9];
    for (int i = 0; i < 100; ++i)
        for (int j = 0; j < 100; ++j)
            for (int k = 0; k < 100; ++k) a[(i * 100 + j) * 100 + k] = i * 1000000 + j * 1000 + k;
    int psize = 0, pos = 0, errs = 0;
    MPI_Pack_size(1, three, MPI_COMM_WORLD, &psize);
    int *oa = ob_alloc(n * sizeof(int));
    void *oe = ob_alloc(sizeof e), *pb = ob_alloc(psize);
    ob_put(oa, a, n * sizeof(int));
    errs += MPI_Pack(oa + (0 * 100 + 2) * 100 + 1, 1, three, pb, psize, &pos, MPI_COMM_WORLD) != MPI_SUCCESS;
    pos = 0;
    errs += MPI_Unpack(pb, psize, &pos, oe, 9 * 9 * 9, MPI_INT, MPI_COMM_WORLD) != MPI_SUCCESS;
    ob_get(e, oe, sizeof e);
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j)
            for (int k = 0; k < 9; ++k) errs += chk(e[i][j][k] == a[(i * 100 + j + 2) * 100 + k * 2 + 1]);
    ob_free(oa);
    ob_free(oe);
    ob_free(pb);
    free(a);
    MPI_Type_free(&three);
    MPI_Type_free(&two);
    MPI_Type_free(&one);
    return errs;
}

/* vecblklen.c:27-80 / hvecblklen.c: 59 chars resized to a 64-byte extent, tiled 16 x 16 by a
 * (h)vector whose block equals its stride; after the round trip every element's 59 bytes are
 * back and its 5 padding bytes keep the fill */
static int blklen_case(int hvec) {
    MPI_Datatype ot, ot2, t;
    MPI_Type_contiguous(59, MPI_CHAR, &ot);
    MPI_Type_create_resized(ot, 0, 64, &ot2);
    if (hvec) MPI_Type_create_hvector(16, 16, 16 * 64, ot2, &t);
    else MPI_Type_vector(16, 16, 16, ot2, &t);
    MPI_Type_commit(&t);
    const int sz = 16 * 16 * 64;
    char *in = malloc(sz), *out = malloc(sz);
    for (int i = 0; i < sz; ++i) in[i] = (char)(i % 64);
    int errs = pack_roundtrip(in, sz, 1, t, 0xff, out, NULL, NULL);
    for (int e = 0; e < 256; ++e)
        for (int k = 0; k < 64; ++k) errs += chk(out[e * 64 + k] == (k < 59 ? (char)k : (char)-1));
    free(in);
    free(out);
    MPI_Type_free(&t);
    MPI_Type_free(&ot2);
    MPI_Type_free(&ot);
    return errs;
}
static int t_vecblklen(void) { return blklen_case(0); }
static int t_hvecblklen(void) { return blklen_case(1); }

/* zeroblks.c:25-60: indexed blocks {0 at 0, 40 at 20}: ints 20..59 travel, 0..19 keep -1 */
static int t_zeroblks(void) {
    int bl[2] = {0, 40}, ds[2] = {0, 20}, s[60], r[60];
    MPI_Datatype t;
    MPI_Type_indexed(2, bl, ds, MPI_INT, &t);
    MPI_Type_commit(&t);
    for (int i = 0; i < 60; ++i) s[i] = i;
    int errs = pack_roundtrip(s, sizeof s, 1, t, 0xff, r, NULL, NULL);
    for (int i = 0; i < 60; ++i) errs += chk(r[i] == (i < 20 ? -1 : i));
    MPI_Type_free(&t);
    return errs;
}

/* zero-blklen-vector.c: a vector whose blocks are empty moves nothing */
static int t_zero_blklen_vector(void) {
    MPI_Datatype t;
    MPI_Type_vector(4, 0, 3, MPI_DOUBLE, &t);
    MPI_Type_commit(&t);
    int sz = -1, errs = 0;
    MPI_Type_size(t, &sz);
    errs += chk(sz == 0);
    double a[12], img[12];
    for (int i = 0; i < 12; ++i) a[i] = 0.5 + i;
    int psz = -1;
    errs += pack_roundtrip(a, sizeof a, 1, t, 0, img, NULL, &psz);
    errs += chk(psz == 0);
    for (int i = 0; i < 12; ++i) errs += chk(img[i] == 0.0);
    MPI_Type_free(&t);
    return errs;
}

/* unpack.c:45-100: indexed({1,2},{0,2}) of indexed({1,2},{0,2}, CHAR), count 2, unpacked from
 * 'a', 'b', ... into a '_'-filled buffer: the letters land on the type map's byte offsets
 * (inner map 0, 2, 3 with extent 4; outer blocks at 0 and 2 inner extents; extent 16) */
static int t_unpack_nested_indexed(void) {
    int bl[2] = {1, 2}, ds[2] = {0, 2};
    MPI_Datatype in, t;
    MPI_Type_indexed(2, bl, ds, MPI_CHAR, &in);
    MPI_Type_commit(&in);
    MPI_Type_indexed(2, bl, ds, in, &t);
    MPI_Type_free(&in);
    MPI_Type_commit(&t);
    int sz = 0, errs = 0;
    MPI_Aint lb = 0, ext = 0;
    MPI_Type_size(t, &sz);
    MPI_Type_get_extent(t, &lb, &ext);
    errs += chk(sz == 9 && ext == 16);
    static const int inner[3] = {0, 2, 3}, outer[3] = {0, 8, 12};  /* outer: disp 0, then 2 x 4 */
    char want[32], img[32], letters[18];
    memset(want, '_', sizeof want);
    int l = 0;
    for (int e = 0; e < 2; ++e)
        for (int o = 0; o < 3; ++o)
            for (int k = 0; k < 3; ++k) want[e * 16 + outer[o] + inner[k]] = (char)('a' + l++);
    for (int i = 0; i < 18; ++i) letters[i] = (char)('a' + i);
    char *om = ob_alloc(32), *op = ob_alloc(18);
    memset(img, '_', 32);
    ob_put(om, img, 32);
    ob_put(op, letters, 18);
    int pos = 0;
    errs += MPI_Unpack(op, 18, &pos, om, 2, t, MPI_COMM_SELF) != MPI_SUCCESS;
    errs += chk(pos == 18);
    ob_get(img, om, 32);
    errs += chk(memcmp(img, want, 32) == 0);
    ob_free(om);
    ob_free(op);
    MPI_Type_free(&t);
    return errs;
}

/* structpack2.c:30-100: struct {int; char} (extent = sizeof, padded), contiguous(10, it) */
struct ic {
    int i;
    char c;
};
static int t_structpack2(void) {
    int bl[2] = {1, 1};
    MPI_Aint ds[2] = {0, sizeof(int)};
    MPI_Datatype ts[2] = {MPI_INT, MPI_CHAR}, st, con;
    MPI_Type_create_struct(2, bl, ds, ts, &st);
    MPI_Type_commit(&st);
    MPI_Type_contiguous(10, st, &con);
    MPI_Type_commit(&con);
    MPI_Aint lb = 0, ext = 0;
    int sz = 0, errs = 0;
    MPI_Type_get_extent(st, &lb, &ext);
    MPI_Type_size(con, &sz);
    errs += chk(ext == sizeof(struct ic) && sz == 10 * 5);
    struct ic s[10], r[10];
    memset(s, 0, sizeof s);
    for (int j = 0; j < 10; ++j) {
        s[j].i = j;
        s[j].c = (char)('a' + j);
    }
    errs += pack_roundtrip(s, sizeof s, 1, con, 0, r, NULL, NULL);
    for (int j = 0; j < 10; ++j) errs += chk(r[j].i == j && r[j].c == 'a' + j);
    MPI_Type_free(&con);
    MPI_Type_free(&st);
    return errs;
}

/* localpack.c:30-75: three values packed one after another into one buffer and unpacked in
 * the same order (positions advance by each type's size) */
static int t_localpack(void) {
    const int n = 10;
    const double a = 1.1, b = 2.2;
    int errs = 0, pos = 0;
    char *pb = ob_alloc(64);
    int *on = ob_alloc(sizeof(int));
    double *oa = ob_alloc(sizeof(double)), *obb = ob_alloc(sizeof(double));
    ob_put(on, &n, sizeof n);
    ob_put(oa, &a, sizeof a);
    ob_put(obb, &b, sizeof b);
    errs += MPI_Pack(on, 1, MPI_INT, pb, 64, &pos, MPI_COMM_WORLD) != MPI_SUCCESS;
    errs += chk(pos == 4);
    errs += MPI_Pack(oa, 1, MPI_DOUBLE, pb, 64, &pos, MPI_COMM_WORLD) != MPI_SUCCESS;
    errs += MPI_Pack(obb, 1, MPI_DOUBLE, pb, 64, &pos, MPI_COMM_WORLD) != MPI_SUCCESS;
    errs += chk(pos == 20);
    const int size = pos;
    const int zi = 0;
    const double zd = 0;
    ob_put(on, &zi, sizeof zi);
    ob_put(oa, &zd, sizeof zd);
    ob_put(obb, &zd, sizeof zd);
    pos = 0;
    errs += MPI_Unpack(pb, size, &pos, on, 1, MPI_INT, MPI_COMM_WORLD) != MPI_SUCCESS;
    errs += MPI_Unpack(pb, size, &pos, oa, 1, MPI_DOUBLE, MPI_COMM_WORLD) != MPI_SUCCESS;
    errs += MPI_Unpack(pb, size, &pos, obb, 1, MPI_DOUBLE, MPI_COMM_WORLD) != MPI_SUCCESS;
    int gn = 0;
    double ga = 0, gb = 0;
    ob_get(&gn, on, sizeof gn);
    ob_get(&ga, oa, sizeof ga);
    ob_get(&gb, obb, sizeof gb);
    errs += chk(gn == 10 && ga == 1.1 && gb == 2.2 && pos == 20);
    ob_free(pb);
    ob_free(on);
    ob_free(oa);
    ob_free(obb);
    return errs;
}

/* pairtype-pack.c:60-110: 16 MPI_SHORT_INT pairs round-trip through a buffer zeroed between
 * pack and unpack; the pairs come back and the padding between short and int stays zero */
struct si {
    short a;
    int b;
};
static int t_pairtype_pack(void) {
    struct si s[16], r[16];
    memset(s, 0, sizeof s);
    for (int i = 0; i < 16; ++i) {
        s[i].a = (short)(i * 2);
        s[i].b = i * 2 + 1;
    }
    int errs = pack_roundtrip(s, sizeof s, 16, MPI_SHORT_INT, 0, r, NULL, NULL);
    for (int i = 0; i < 16; ++i) {
        errs += chk(r[i].a == (short)(i * 2) && r[i].b == i * 2 + 1);
        const unsigned char *pad = (const unsigned char *)&r[i] + sizeof(short);
        for (size_t k = 0; k < offsetof(struct si, b) - sizeof(short); ++k) errs += chk(pad[k] == 0);
    }
    return errs;
}

/* contig-zero-count.c / blockindexed-zero-count.c / struct-zero-count.c: types of zero
 * elements have size 0 and pack nothing */
static int t_zero_count_types(void) {
    int errs = 0, zero = 0, sz = -1;
    MPI_Aint lb = -1, ext = -1;
    MPI_Datatype t[3];
    int bl[1] = {1};
    MPI_Aint ds[1] = {0};
    MPI_Datatype ts[1] = {MPI_INT};
    MPI_Type_contiguous(0, MPI_INT, &t[0]);
    MPI_Type_create_indexed_block(0, 1, &zero, MPI_INT, &t[1]);
    MPI_Type_create_struct(0, bl, ds, ts, &t[2]);
    for (int k = 0; k < 3; ++k) {
        MPI_Type_commit(&t[k]);
        MPI_Type_size(t[k], &sz);
        MPI_Type_get_extent(t[k], &lb, &ext);
        errs += chk(sz == 0 && ext == 0);
        int v[4] = {7, 8, 9, 10}, img[4], psz = -1;
        errs += pack_roundtrip(v, sizeof v, 3, t[k], 0, img, NULL, &psz);
        errs += chk(psz == 0);
        MPI_Type_free(&t[k]);
    }
    return errs;
}

static const struct {
    const char *name;
    int (*fn)(void);
} kCases[] = {
    {"simple_pack_nested", t_simple_pack_nested},
    {"simple_pack_contig_vector", t_simple_pack_contig_vector},
    {"transpose_pack", t_transpose_pack},
    {"triangular_pack", t_triangular_pack},
    {"slice_pack", t_slice_pack},
    {"vecblklen", t_vecblklen},
    {"hvecblklen", t_hvecblklen},
    {"zeroblks", t_zeroblks},
    {"zero_blklen_vector", t_zero_blklen_vector},
    {"unpack_nested_indexed", t_unpack_nested_indexed},
    {"structpack2", t_structpack2},
    {"localpack", t_localpack},
    {"pairtype_pack", t_pairtype_pack},
    {"zero_count_types", t_zero_count_types},
};

int main(int argc, char **argv) {
    if (argc < 2 || (strcmp(argv[1], "host") && strcmp(argv[1], "device"))) {
        fprintf(stderr, "usage: dt_suite {host|device} [case ...]\n");
        return 2;
    }
    g_dev = !strcmp(argv[1], "device");
    MPI_Init(&argc, &argv);
    MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN);
    int total = 0, ran = 0;
    for (size_t k = 0; k < sizeof kCases / sizeof kCases[0]; ++k) {
        int wanted = argc <= 2;
        for (int a = 2; a < argc; ++a) wanted |= !strcmp(argv[a], kCases[k].name);
        if (!wanted) continue;
        const int errs = kCases[k].fn();
        printf("%s %s %d\n", argv[1], kCases[k].name, errs);
        fflush(stdout);
        total += errs;
        ++ran;
    }
    printf("%s TOTAL %d cases %d\n", argv[1], total, ran);
    MPI_Finalize();
    return total ? 1 : 0;
}
