/*
 * mv2h.h — C-ABI between the MPI entry points (C glue) and the MI355X HIP
 * layer of mvapich2_amd.  Plain pointers and sizes only; no HIP or torch
 * types appear in these signatures (`stream` is a hipStream_t passed as
 * void*, NULL = the library's internal stream).
 *
 * Every entry point is synchronous with respect to the caller (MPI blocking
 * semantics): on return the result is complete in device memory — except the
 * stream-ordered *_enqueue calls, which complete in the order of their stream.
 * Return value is MPI_SUCCESS (0) or an MPI error class.
 *
 * Reference interfaces each entry point replaces (MVAPICH2 2.3.7):
 *   mv2h_reduce_local   MPIR_Reduce_local_impl        src/mpi/coll/reduce_local.c:36-173
 *                       (host op kernels              src/mpi/coll/op*.c, oputil.h:50-57)
 *   mv2h_op_check       MPIR_Op_check_dtype_table     src/mpi/coll/allreduce.c:102-109
 *   mv2h_allreduce      MPIR_Allreduce_MV2            src/mpi/coll/allreduce_osu.c:3720
 *                       -> index_tuned_intra_MV2      allreduce_osu.c:3015-3420
 *   mv2h_reduce         MPIR_Reduce_MV2               src/mpi/coll/reduce_osu.c:2709
 *   mv2h_reduce_scatter MPIR_Reduce_scatter_MV2       src/mpi/coll/red_scat_osu.c:1771
 *   mv2h_allgather      MPIR_Allgather_MV2            src/mpi/coll/allgather_osu.c:2593
 *   mv2h_bcast          MPIR_Bcast_MV2                src/mpi/coll/bcast_osu.c:3347
 *   mv2h_pack_strided   MPID_Segment_pack_device      src/mpid/ch3/channels/mrail/src/gen2/ibv_cuda_util.c:623
 *                       pack_unpack_vector_kernel     src/mpid/ch3/channels/mrail/src/cuda/pack_unpack.cu:419
 *   mv2h_is_device_ptr  is_device_buffer              ibv_cuda_util.c:819
 */
#ifndef MV2H_H_INCLUDED
#define MV2H_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Reduction order used by the n-input device reduction.
 * Each reproduces the operand order of one MV2 host algorithm bit-for-bit. */
enum mv2h_order {
    MV2H_ORDER_LINEAR = 0,    /* ((x0 op x1) op x2) ... : two-level reduce_shmem, allreduce_osu.c:1569-1583 */
    MV2H_ORDER_BUTTERFLY = 1, /* recursive halving / doubling with non-pof2 fold, allreduce_osu.c:455-947 */
};

/* ---- library / device bookkeeping ---- */
const char *mv2h_version(void);
int mv2h_device_count(void);
int mv2h_is_device_ptr(const void *ptr);
int mv2h_malloc(void **ptr, size_t bytes);
int mv2h_free(void *ptr);
int mv2h_memcpy_htod(void *dst, const void *src, size_t bytes);
int mv2h_memcpy_dtoh(void *dst, const void *src, size_t bytes);
int mv2h_memcpy_dtod(void *dst, const void *src, size_t bytes);
int mv2h_memset(void *dst, int value, size_t bytes);
int mv2h_device_synchronize(void);

/* ---- datatypes / op table ---- */
int mv2h_dtype_info(int dtype, size_t *size, size_t *extent);
int mv2h_op_check(int op, int dtype);

/* ---- part (1): the MPI_Op reduction layer ---- */
int mv2h_reduce_local(const void *in, void *inout, size_t count, int dtype, int op, void *stream);
/* dst = reduce(srcs[0..nsrc-1]) in `order`; owner = newrank whose subtree is the left
 * operand (butterfly only).  srcs may be peer (IPC-mapped) pointers. */
int mv2h_reduce_n(const void *const *srcs, int nsrc, void *dst, size_t count, int dtype, int op,
                  int order, int owner, void *stream);

/* ---- part (2): device collectives over COMM_WORLD (one process per GPU) ---- */
int mv2h_allreduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op,
                   void *stream);
int mv2h_reduce(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op, int root,
                void *stream);
int mv2h_reduce_scatter(const void *sendbuf, void *recvbuf, const size_t *recvcounts, int dtype,
                        int op, void *stream);
int mv2h_allgather(const void *sendbuf, void *recvbuf, size_t bytes_per_rank, void *stream);
int mv2h_bcast(void *buffer, size_t bytes, int root, void *stream);
int mv2h_barrier(void);

/* ---- stream-ordered collectives (SURVEY §8(f) rank 3 "stream-ordered variants") ----
 * Same selection, reduction orders and kernels as the calls above, launched on `stream`
 * (a hipStream_t, required) after every collective this process issued before on any
 * stream, and returning without waiting: work queued behind them on `stream` sees the
 * result.  Device buffers and predefined ops only (E_ARG otherwise).  Buffers must stay
 * valid until the stream reaches the call.  A peer that never arrives makes the kernel
 * give up after MV2AMD_TIMEOUT_S and raise the error that mv2h_enqueue_check (or the next
 * blocking call) returns once the stream has been synchronised.  A stream that is being
 * captured into a HIP graph is refused (E_UNSUPPORTED): a replay would reuse the captured
 * call's flag epochs. */
int mv2h_allreduce_enqueue(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op,
                           void *stream);
int mv2h_reduce_enqueue(const void *sendbuf, void *recvbuf, size_t count, int dtype, int op,
                        int root, void *stream);
int mv2h_reduce_scatter_enqueue(const void *sendbuf, void *recvbuf, const size_t *recvcounts,
                                int dtype, int op, void *stream);
int mv2h_allgather_enqueue(const void *sendbuf, void *recvbuf, size_t bytes_per_rank, void *stream);
int mv2h_bcast_enqueue(void *buffer, size_t bytes, int root, void *stream);
int mv2h_copy_enqueue(void *dst, const void *src, size_t bytes, void *stream);
int mv2h_enqueue_check(void);

/* ---- nonblocking collectives (MPI_Iallreduce family, reference iallreduce_osu.c) ----
 * Between mv2h_defer_begin() and mv2h_defer_end(&ticket) the device collectives above
 * return right after their kernel is enqueued instead of waiting for it.  ticket > 0:
 * the call's completion word; ticket == 0: the call already completed (host-staged or
 * copy-back paths complete at initiation, which MPI allows).  Tickets complete in issue
 * order (one stream).  mv2h_wait_ticket blocks; mv2h_test_ticket sets *done.  Both return
 * the collective's error class (e.g. a peer timeout), 0 on success. */
/* ---- point-to-point (runtime/p2p.cpp; reference ch3 eager/IPC path, ch3u_recvq.c matching) ----
 * Byte messages between ranks (global ranks, MPI_COMM_WORLD numbering); buffers may be device
 * or host memory.  Within a node a send completes when its last chunk is in the receiver's
 * arena; to a rank on another node (the rank mesh, TCP) when its bytes are in the socket
 * (buffer reusable either way).  A receive completes when the matched message is in `buf`
 * (E_TRUNCATE if it was longer than cap: the first cap bytes are delivered).  Matching:
 * posting order against arrival order, MV2H_ANY_SOURCE / MV2H_ANY_TAG wildcards (application
 * tags >= 0 only), non-overtaking per (source, tag).  Progress happens inside every
 * isend/irecv/test/wait call. */
#define MV2H_ANY_SOURCE (-2)
#define MV2H_ANY_TAG (-1)
int mv2h_isend(const void *buf, size_t bytes, int dest, int tag, unsigned long long *req);
int mv2h_irecv(void *buf, size_t cap, int source, int tag, unsigned long long *req);
int mv2h_p2p_test(unsigned long long req, int *done, int *source, int *tag, size_t *bytes);
int mv2h_p2p_wait(unsigned long long req, int *source, int *tag, size_t *bytes);
/* progress, then *done = whether `req` has completed, without completing it (MPI_Testall's
 * all-or-nothing check, MPI-3.1 §3.7.5) */
int mv2h_p2p_peek(unsigned long long req, int *done);
int mv2h_p2p_progress(void);

int mv2h_defer_begin(void);
int mv2h_defer_end(unsigned long long *ticket);
int mv2h_wait_ticket(unsigned long long ticket);
int mv2h_test_ticket(unsigned long long ticket, int *done);

/* ---- part (3): strided pack / unpack (MPI_Type_vector family) ----
 * pack:   dst[i*blk + j] = src[i*stride + j],  i < nblocks, j < blk  (bytes)
 * unpack: dst[i*stride + j] = src[i*blk + j] */
int mv2h_pack_strided(const void *src, void *dst, size_t nblocks, size_t blk_bytes,
                      size_t stride_bytes, void *stream);
int mv2h_unpack_strided(const void *src, void *dst, size_t nblocks, size_t blk_bytes,
                        size_t stride_bytes, void *stream);
/* Any flattened layout (pair types, indexed types, vectors with count > 1, nested types):
 * one element = nseg byte segments (offs[s], lens[s]) in pack order, `count` elements
 * `extent` bytes apart; packed element e holds its segments back to back at e * sum(lens).
 *   pack:   packed[e*size + pos(s) + b] = src[e*extent + offs[s] + b]
 *   unpack: the inverse; bytes outside the segments are never written.
 * Replaces Segment_pack / Segment_unpack (segment_packunpack.c:70/96, m2m callbacks
 * :124-388) and MPID_Segment_pack_device / _unpack_device (ibv_cuda_util.c:623 / :720). */
int mv2h_pack_segments(const void *src, void *dst, size_t count, size_t extent,
                       const int64_t *offs, const int64_t *lens, int nseg, int unpack,
                       void *stream);

/* ---- reduction-order plans (host only: no GPU needed) ----
 * The algorithm MVAPICH2 2.3.7 selects for a one-node collective and the
 * reduction order it gives each element, as register programs:
 * registers w[j] = rank j's operand; step s: w[dst[s]] = uop(in = w[src[s]],
 * inout = w[dst[s]]); result w[res].  Element e uses p[min(e / blk, nprog-1)].
 * Replaces the selection in MPIR_Allreduce_index_tuned_intra_MV2
 * (allreduce_osu.c:3015-3420), MPIR_Reduce_index_tuned_intra_MV2
 * (reduce_osu.c:2391-2660) and MPIR_Reduce_scatter_MV2 (red_scat_osu.c:1771). */
typedef struct {
    uint8_t nsteps, res;
    uint8_t dst[7];
    uint8_t src[7];
} mv2h_prog;
typedef struct {
    int32_t nprog, pad;
    uint64_t blk;
    mv2h_prog p[8];
} mv2h_progset;
enum mv2h_coll {
    MV2H_COLL_ALLREDUCE = 0,      /* count; in_place */
    MV2H_COLL_REDUCE = 1,         /* count; root */
    MV2H_COLL_REDUCE_SCATTER = 2, /* counts[n] */
    MV2H_COLL_ALLREDUCE_RS = 3,   /* pt2pt_rs forced (ring wrapper remainder / IN_PLACE body) */
};
/* opkind: 0 builtin, 1 commutative user op, 2 non-commutative user op.
 * *algo: 0 none, 1 shmem_linear, 2 pt2pt_rs, 3 pt2pt_rd, 4 ring_wrapper,
 * 5 topo_tree, 6 two_level_p2p, 7 binomial, 8 knomial, 9 redscat_gather,
 * 10 rs_ring, 11 rs_rec_halving, 12 rs_pairwise, 13 rs_basic, 14 reduce_topo,
 * 15 rs_noncomm_pof2, 16 rs_noncomm_rd (non-commutative user ops' reduce-scatter).
 * *unpinned = 1 when the reference's own result depends on message arrival. */
int mv2h_plan(int coll, int n, int rank, int root, size_t count, const size_t *counts, int dtype, int opkind,
              int in_place, int *algo, int *inner, int *unpinned, mv2h_progset *ps);
/* Several nodes: the allreduce tuning-table entry for ppn ranks per node, gsize ranks and nbytes
 * (allreduce_osu.c:3162-3290 over every numproc entry of the default 1 / 2 / 16-ppn tables).
 * Returns 0 for a two-level entry (*intra: 0 the node's own selection, 1 reduce_shmem,
 * 2 reduce_p2p, 3 pt2pt_rs, 4 pt2pt_rd; *inter: 2 pt2pt_rs, 3 pt2pt_rd), 2 / 3 for a flat
 * pt2pt_rs / pt2pt_rd over every rank. */
int mv2h_mn_allreduce_table(int ppn, int gsize, long nbytes, int *intra, int *inter);
/* MPIR_Reduce_scatter_MV2's blocking choice for a commutative op over n ranks and nbytes in all
 * (red_scat_osu.c:1859-1893, the default table of red_scat_tuning.c): *algo codes of mv2h_plan
 * (10 rs_ring, 11 rs_rec_halving, 12 rs_pairwise, 13 rs_basic). */
int mv2h_reduce_scatter_table(int n, long nbytes);
/* The expression of rank me's block of the non-commutative reduce-scatter over n ranks (the host
 * evaluates it above 8 ranks): node i is rank leaf[i]'s operand when leaf[i] >= 0, else
 * uop(in = node b[i], inout = node a[i]); *root the result's node.  Returns the node count, or minus
 * the count needed when cap is too small. */
int mv2h_rs_noncomm_expr(int n, int me, int pof2_equal, int *leaf, int *a, int *b, int cap, int *root);
/* The message schedules the host evaluates for a user op above 8 ranks (mpi/user_coll.cpp BigEval),
 * run on n int32 operands of count elements each (ops: operand r at ops + r * count) with the fixed
 * function inout = 2 in + 3 inout; commute as the op's flag.  Writes rank me's (MPI_Reduce: the
 * root's) result to out: recursive doubling (allreduce_osu.c:455-600), pt2pt_rs (:852-1000),
 * binomial (reduce_osu.c:577-663), knomial with factor k (:1639-1837), redscat_gather (:718-1100),
 * the reduce-scatter's recursive halving / pairwise / ring over one block (red_scat_osu.c:428-1180),
 * the allreduce ring's chunk me (allreduce_osu.c:3916-3968), and the non-commutative reduce-scatter's
 * expression for block me with equal counts (red_scat_osu.c:132-290 / :1478-1722).  Needs no GPU.
 * Test hook. */
enum mv2h_sched_form {
    MV2H_SCHED_RD = 0,
    MV2H_SCHED_PT2PT_RS = 1,
    MV2H_SCHED_BINOMIAL = 2,
    MV2H_SCHED_KNOMIAL = 3,
    MV2H_SCHED_REDSCAT_GATHER = 4,
    MV2H_SCHED_RS_HALVING = 5,
    MV2H_SCHED_RS_PAIRWISE = 6,
    MV2H_SCHED_RS_RING = 7,
    MV2H_SCHED_RING_CHUNK = 8,
    MV2H_SCHED_RS_NONCOMM = 9  /* the non-commutative reduce-scatter's expression for rank me's block */
};
int mv2h_host_sched_eval(int form, int n, int me, int root, int k, int count, int commute, const int32_t *ops,
                         int32_t *out);
/* Several nodes: MPI_Reduce's tuning-table cell (reduce_osu.c:2516-2620, the default tables of
 * reduce_tuning.c:1563-1649, CMA or not as MV2_SMP_USE_CMA says): *two_level = 1 for
 * MPIR_Reduce_two_level_helper_MV2, *inter the leaders' (or flat) algorithm and *intra the node step
 * (mv2h_plan algo codes: 1 shmem, 7 binomial, 8 knomial, 9 redscat_gather), *k the knomial factor.
 * Returns the table entry index (comm_size_index), or an error class. */
int mv2h_mn_reduce_table(int ppn, int gsize, long nbytes, int *two_level, int *inter, int *intra, int *k);
/* Several nodes: the route a builtin-op call takes (coll 0 MPI_Allreduce, 1 MPI_Reduce, 2
 * MPI_Reduce_scatter; nbc: enum mv2h_nbc): 0 two-level, 1 flat ring over every rank, 2 a flat
 * algorithm as per-element programs (up to 8 ranks), 3 its message schedule over the rank channels
 * (up to 64 ranks), 4 the two-level structure standing in above 64 ranks (fp order unpinned),
 * 5 the basic reduce-scatter.  *rem_route: the ring wrapper's remainder's route, -1 for none.
 * 12 (MPI_ERR_ARG's class) for a shape that is not ppn ranks on each of gsize / ppn nodes. */
int mv2h_mn_route(int coll, int ppn, int gsize, long nbytes, size_t count, int in_place, int nbc, int *rem_route);
/* Nonblocking initiation: between mv2h_nbc_begin(kind) and mv2h_nbc_end() on this thread
 * the reducing collectives take the reference's nonblocking selection (MPIR_Iallreduce_MV2,
 * MPIR_Ireduce_MV2, MPIR_Ireduce_scatter_MV2, MPICH MPIR_Ireduce_scatter_block_intra) and
 * its reduction order instead of the blocking one. */
enum mv2h_nbc {
    MV2H_NBC_NONE = 0,
    MV2H_NBC_IALLREDUCE = 1,
    MV2H_NBC_IREDUCE = 2,
    MV2H_NBC_IREDUCE_SCATTER = 3,
    MV2H_NBC_IREDUCE_SCATTER_BLOCK = 4
};
int mv2h_nbc_begin(int kind);
int mv2h_nbc_end(void);
int mv2h_knobs_reload(void);
/* Intra-node topology levels of the topology-aware shm tree (create_2level_comm.c:
 * 916-986): colors[l * n + r] = local rank r's cluster id at level l (its NUMA node, then its
 * socket), which MPI_Init derives from every rank's CPU binding; set = override for the plans
 * computed afterwards (tests, tools).  nlevels <= 4, n <= 8. */
int mv2h_set_topology(int nlevels, const int *colors, int n);
int mv2h_get_topology(int *nlevels, int *colors, int n);
/* dst = reduce(srcs[0..nsrc-1]) by the programs of *ps (single GPU; order tests) */
int mv2h_reduce_n_prog(const void *const *srcs, int nsrc, void *dst, size_t count, int dtype, int op,
                       const mv2h_progset *ps, void *stream);

/* ---- runtime (bootstrap for COMM_WORLD) ---- */
int mv2h_init(void);
int mv2h_finalize(void);
int mv2h_rank(void);
int mv2h_size(void);
int mv2h_local_rank(void);

/* ---- measurement hooks (bench.py): HIP-event timing of the last kernel ---- */
int mv2h_timing_enable(int on);
double mv2h_last_kernel_ms(void);
int mv2h_set_tuning(const char *key, long value);
/* runtime facts: "nshare" (most ranks sharing one GPU), "device", "cus", "light_release", "oneshot_max",
 * "pipe_grid" / "pipe_sub" (pipelined kernels' tiling), "pipe_tuned" (1: chosen by the MPI_Init
 * autotune), "tune_n" and per candidate k "tune_grid_<k>", "tune_sub_<k>", "tune_us_<k>" (max over ranks),
 * "init_us" / "hip_init_us" / "code_load_us" / "selftest_us" / "autotune_us" (this rank's MPI_Init
 * wall time and its parts), "selftest_calls" (collective calls MPI_Init's self-test checked),
 * "call_allocs" (device allocations made inside MPI calls: scratch growth, pooled temporaries),
 * "hw_queues_set" (GPU_MAX_HW_QUEUES set before HIP started; negative: wanted, but HIP was already
 * running) */
int mv2h_get_info(const char *key, long *value);

#ifdef __cplusplus
}
#endif

#endif /* MV2H_H_INCLUDED */
