// orders.h — which MV2 algorithm a one-node collective runs, and the
// reduction order that algorithm gives every element (as Prog programs).
//
// The reference picks an algorithm per call from size thresholds, MV2_*
// knobs and tuning tables (MPIR_Allreduce_index_tuned_intra_MV2
// allreduce_osu.c:3015-3420, MPIR_Reduce_index_tuned_intra_MV2
// reduce_osu.c:2391-2660, MPIR_Reduce_scatter_MV2 red_scat_osu.c:1771-1900),
// and the fp result depends on that algorithm's operand order.  This module
// restates the selection for one node (shmem_coll_ok, is_uniform, blocked
// placement, one topology level: see DESIGN.md §4) and turns each algorithm
// into per-element programs by a symbolic run of its message schedule: the
// device kernels then evaluate the same binary tree in registers.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../coll/kernels.h"

namespace mv2 {

enum Algo : int {
    ALG_NONE = 0,            // one rank / REPLACE / NO_OP: no reduction order
    ALG_SHMEM_LINEAR = 1,    // reduce_shmem / MPIR_Reduce_shmem_MV2: ((x0 . x1) . x2) ...
    ALG_PT2PT_RS = 2,        // MPIR_Allreduce_pt2pt_rs_MV2 (allreduce_osu.c:633)
    ALG_PT2PT_RD = 3,        // MPIR_Allreduce_pt2pt_rd_MV2 (:360), also pt2pt_rs with count < pof2
    ALG_RING = 4,            // MPIR_Allreduce_pt2pt_ring_wrapper_MV2 (:3758)
    ALG_TOPO_TREE = 5,       // MPIR_Allreduce_topo_aware_hierarchical_MV2 (:2272) -> mv2_shm_tree_reduce
    ALG_TWO_LEVEL_P2P = 6,   // two-level with intra reduce_p2p: MPIR_Reduce_MV2 to local rank 0 (:1616)
    ALG_BINOMIAL = 7,        // MPIR_Reduce_binomial_MV2 (reduce_osu.c:425)
    ALG_KNOMIAL = 8,         // MPIR_Reduce_knomial_MV2 (:1639)
    ALG_REDSCAT_GATHER = 9,  // MPIR_Reduce_redscat_gather_MV2 (:718)
    ALG_RS_RING = 10,        // MPIR_Reduce_scatter_ring(_2lvl) (red_scat_osu.c:1026/1190)
    ALG_RS_REC_HALVING = 11, // MPIR_Reduce_scatter_Rec_Halving_MV2 (:428)
    ALG_RS_PAIRWISE = 12,    // MPIR_Reduce_scatter_Pair_Wise_MV2 (:786)
    ALG_RS_BASIC = 13,       // MPIR_Reduce_Scatter_Basic_MV2 (:300): MPIR_Reduce_MV2 to 0 + scatter
    ALG_REDUCE_TOPO = 14,    // MPIR_Reduce_topo_aware_hierarchical_MV2 (reduce_osu.c:206)
    ALG_RS_NONCOMM_POF2 = 15,// MPIR_Reduce_scatter_noncomm_MV2 (red_scat_osu.c:132): pof2, equal counts
    ALG_RS_NONCOMM_RD = 16,  // MPIR_Reduce_scatter_non_comm_MV2's recursive doubling (:1478)
    ALG_COUNT
};

// MV2_* knobs that move the one-node selection, parsed like the reference
// (ch3_shmem_coll.c MV2_Read_env_vars; atoi unless the reference uses
// user_val_to_bytes).  Defaults: ch3_shmem_coll.c:283-541, coll_shmem.h:35/191,
// mpiimpl.h:3954, ch3_smp_progress.c:221.
struct Knobs {
    int32_t enable_shmem_collectives;   // MV2_USE_SHARED_MEM (1)
    int32_t enable_shmem_allreduce;     // MV2_USE_SHMEM_ALLREDUCE (1)
    int32_t enable_shmem_reduce;        // MV2_USE_SHMEM_REDUCE (1)
    int32_t enable_skip_search;         // MV2_ENABLE_SKIP_TUNING_TABLE_SEARCH (1)
    int32_t coll_skip_thr;              // MV2_COLL_SKIP_TABLE_THRESHOLD (1024, atoi)
    int32_t allred_skip_small;          // MV2_ENABLE_ALLREDUCE_SKIP_SMALL_MESSAGE_TUNING_TABLE_SEARCH (1)
    int32_t allred_skip_large;          // MV2_ENABLE_ALLREDUCE_SKIP_LARGE_MESSAGE_TUNING_TABLE_SEARCH (1)
    int32_t enable_topo;                // MV2_ENABLE_TOPO_AWARE_COLLECTIVES (1; 0 if socket-aware is enabled)
    int32_t use_topo_allreduce;         // MV2_USE_TOPO_AWARE_ALLREDUCE (1)
    int32_t topo_allred_min, topo_allred_max;   // MV2_TOPO_AWARE_ALLREDUCE_{MIN,MAX}_MSG (1, 2048)
    int32_t topo_allred_ppn;            // mv2_topo_aware_allreduce_ppn_threshold (1)
    int32_t use_topo_reduce;            // MV2_USE_TOPO_AWARE_REDUCE (0)
    int32_t topo_red_min, topo_red_max; // MV2_TOPO_AWARE_REDUCE_{MIN,MAX}_MSG (1, 2048)
    int32_t topo_red_ppn;               // MV2_TOPO_AWARE_REDUCE_PPN_THRESHOLD (1)
    int32_t topo_red_nodes;             // MV2_TOPO_AWARE_REDUCE_NODE_THRESHOLD (1)
    int32_t tree_degree;                // MV2_SHMEM_REDUCE_TREE_DEGREE (4)
    int32_t allred_use_ring;            // MV2_ALLRED_USE_RING (1; flag > 0)
    int32_t pad0;                       // (explicit: the struct is compared bytewise across ranks)
    int64_t allred_ring_thr;            // MV2_ALLREDUCE_RING_ALGO_THRESHOLD (2 MiB, user_val_to_bytes)
    int32_t allred_ring_ppn;            // MV2_ALLREDUCE_RING_ALGO_PPN_THRESHOLD (8)
    int32_t smp_use_cma;                // MV2_SMP_USE_CMA (1): selects the CMA reduce tables
    int32_t use_knomial_reduce;         // MV2_USE_KNOMIAL_REDUCE (1)
    int32_t reduce_inter_k;             // MV2_USE_INTER_KNOMIAL_REDUCE_FACTOR (-1: the table's inter_k_degree)
    int32_t shmem_coll_max_msg;         // MV2_SHMEM_COLL_MAX_MSG_SIZE (32 KiB)
    int32_t shmem_intra_reduce_msg;     // MV2_INTRA_SHMEM_REDUCE_MSG (2048)
    int64_t red_scat_ring_thr;          // MV2_RED_SCAT_RING_ALGO_THRESHOLD (131072, user_val_to_bytes)
    // MPICH cvars of the nonblocking schedules (MPIR_CVAR_*, also MPICH_* env names)
    int32_t reduce_short_msg;           // MPIR_CVAR_REDUCE_SHORT_MSG_SIZE (2048, reduce.c:28-31)
    int32_t pad1;
    int64_t redscat_comm_long;          // MPIR_CVAR_REDSCAT_COMMUTATIVE_LONG_MSG_SIZE (524288, red_scat.c)
};

const Knobs &knobs();  // parsed from the environment on first use
void knobs_reload();   // re-read the environment (tests)

// Intra-node topology levels of the topology-aware collectives.  The reference splits the node's
// communicator level by level (create_intra_node_multi_level_topo_comm, create_2level_comm.c:
// 916-986, with create_intra_node_topo_comm_at_level :666-900): at level l every rank takes its
// own cluster id mv2_intra_node_cluster_at_level[l] (hwloc_bind.c:83) as the split colour — the
// NUMA node it is bound to when the node has several (smpi_identify_my_numa_id :2252-2298), then
// its socket when there are several and its NUMA node is not inside it (smpi_identify_my_sock_id
// :2180-2250); levels past a rank's own count read 0 — and the first rank of each group leads it
// into the next level.  mv2_shm_tree_reduce runs once per level (allreduce_osu.c:2340-2361,
// reduce_osu.c:272-296).  color[l][r] = rank r's cluster id at level l, for l < nlevels.
constexpr int kTopoLevels = 4;
struct Topo {
    int nlevels;
    int color[kTopoLevels][kMaxRanks];
};
const Topo &topo();           // default: no level (one group: the node)
void topo_set(const Topo &t); // MPI_Init (runtime/world.cpp) or a test; invalidates cached plans

// Plan::via: how the reference reached the algorithm (for the MPI_T counters
// of its call chain, runtime/pvars.cpp)
enum : int {
    VIA_RS_ENTRY = 1,          // recursive doubling run inside MPIR_Allreduce_pt2pt_rs_MV2 (:802)
    VIA_TWO_LEVEL_HELPER = 2,  // reduce through MPIR_Reduce_two_level_helper_MV2 (reduce_osu.c:2030)
};

struct Plan {
    int algo;    // Algo
    int inner;   // ALG_TWO_LEVEL_P2P / ALG_RS_BASIC: the MPIR_Reduce_MV2 algorithm inside
    int k;       // knomial factor / shm tree degree
    int unpinned;// 1: the reference result depends on message arrival (knomial Waitany)
    int via;     // VIA_* bits
    int pad;
    ProgSet ps;  // order of every element of this rank's result (global element index)
};

// Kind of op: builtin ops are commutative; user ops are commutative or not
// (MPI_Op_create); several algorithms branch on HANDLE_KIND_BUILTIN and on
// is_commutative.  A program step dst <- src is uop(in = w[src], inout = w[dst])
// for every kind, so a non-commutative order is expressed by which operand
// is the accumulator.
enum OpKind : int { OPK_BUILTIN = 0, OPK_USER_COMM = 1, OPK_USER_NONCOMM = 2 };

// All functions: n ranks on one node, tsize = MPI_Type_size, textent = extent.
// Return 0, or E_INTERN when the order cannot be expressed.  forced: 0 = the
// reference's selection, else an Algo to run (ring wrapper parts).
int plan_allreduce(int n, int me, size_t count, int tsize, int textent, bool in_place, int forced, Plan *out,
                   int opk = OPK_BUILTIN);
// several nodes: the allreduce tuning-table choice (0 two-level, ALG_PT2PT_RS / _RD flat, -1 unknown).
// For a two-level entry *intra / *inter name the entry's node step (MN_INTRA_*) and the leaders'
// algorithm (ALG_PT2PT_RD / ALG_PT2PT_RS) of MPIR_Allreduce_two_level_MV2 (allreduce_osu.c:1687-1800).
enum MnIntra : int {
    MN_INTRA_NODE = 0,    // the node's own one-node selection reads the same table entry (16 ppn)
    MN_INTRA_SHMEM = 1,   // MPIR_Allreduce_reduce_shmem_MV2: ((x0 . x1) . x2) ... at the leader
    MN_INTRA_P2P = 2,     // MPIR_Allreduce_reduce_p2p_MV2: MPIR_Reduce_MV2 to local rank 0 (:1614-1684)
    MN_INTRA_RS = 3,      // MPIR_Allreduce_pt2pt_rs_MV2 over the node's communicator, leader's result
    MN_INTRA_RD = 4,      // MPIR_Allreduce_pt2pt_rd_MV2 over the node's communicator, leader's result
};
int mn_allreduce_table(int ppn, int gsize, long nbytes, int *intra = nullptr, int *inter = nullptr);
int plan_reduce(int n, int me, int root, size_t count, int tsize, int textent, Plan *out, int opk = OPK_BUILTIN);
// several nodes: MPI_Reduce's tuning-table cell (reduce_osu.c:2516-2620) for ppn ranks per node,
// gsize ranks and nbytes: two_level (MPIR_Reduce_two_level_helper_MV2) with the node step `intra`
// (ALG_SHMEM_LINEAR / ALG_BINOMIAL / ALG_KNOMIAL to local rank 0) and the leaders' `inter`
// (ALG_BINOMIAL / ALG_KNOMIAL / ALG_REDSCAT_GATHER), or `inter` flat over every rank; k = the
// knomial factor; entry = comm_size_index
struct MnReduceCell {
    int two_level, inter, intra, k, entry;
};
int mn_reduce_table(int ppn, int gsize, long nbytes, MnReduceCell *c);
// the programs of one reduce algorithm to `root` over n ranks (the steps of the two-level helper
// and the flat algorithms across nodes)
int plan_reduce_forced(int n, int root, size_t count, int algo, int k, Plan *out, bool noncomm = false);
// MPIR_Reduce_binomial_MV2 (reduce_osu.c:425) to `root`, whatever the selection (the leaders' step
// of MPIR_Reduce_two_level_helper_MV2 across nodes)
int plan_binomial(int n, int root, Plan *out, bool noncomm = false);
// MPI_Reduce_scatter's algorithm for a commutative op over n ranks and nbytes in all (ALG_RS_*):
// reduce_scatter_table = the blocking selection, reduce_scatter_algo = the one of the call being
// initiated (nonblocking schedules while nbc_set names one)
int reduce_scatter_table(int n, long nbytes);
int reduce_scatter_algo(int n, long nbytes);
// counts[n] per-rank block counts; elements are indexed over the whole operand
int plan_reduce_scatter(int n, int me, const size_t *counts, int tsize, int textent, Plan *out,
                        int opk = OPK_BUILTIN);
// The expression of rank me's block of MPIR_Reduce_scatter_non_comm_MV2 over any number of ranks
// (more than a program's registers: the host evaluates it, mpi/user_coll.cpp): pof2_equal selects
// MPIR_Reduce_scatter_noncomm_MV2's mirror-permuted halving (red_scat_osu.c:132-290), else the
// recursive doubling (:1478-1722).  nodes[i].leaf >= 0: that rank's operand; else
// uop(in = value of nodes[i].b, inout = value of nodes[i].a).  Returns the root node's index.
struct ExprNode {
    int leaf, a, b;
};
int rs_noncomm_expr(int n, int me, bool pof2_equal, std::vector<ExprNode> &nodes);

// Nonblocking collectives.  While a nonblocking call is being initiated
// (nbc_set(kind) on this thread), plan_allreduce / plan_reduce /
// plan_reduce_scatter restate the nonblocking selection instead of the
// blocking one: MVAPICH2 installs MPIR_Iallreduce_MV2 / MPIR_Ireduce_MV2 /
// MPIR_Ireduce_scatter_MV2 (ch3i_comm.c:38-43, enabled by default,
// ch3_shmem_coll.c:432-441) and MPICH's MPIR_Ireduce_scatter_block_intra.
enum NbcKind : int {
    NBC_NONE = 0,
    NBC_IALLREDUCE = 1,
    NBC_IREDUCE = 2,
    NBC_IREDUCE_SCATTER = 3,
    NBC_IREDUCE_SCATTER_BLOCK = 4,  // also the blocking MPI_Reduce_scatter_block (same MPICH selection)
};
void nbc_set(int kind);
int nbc_kind();

// Several nodes: the schedule of a host-evaluated reduction (user MPI_Op, x87 types) over the job,
// as runtime/coll.cpp restates it for the device path (mn_select, MPIR_Allreduce_two_level_MV2,
// MPIR_Reduce_two_level_helper_MV2, the flat algorithms over every rank).  MN_FLAT: `p` holds this
// rank's programs over the job's ranks (forced: the plan_allreduce / plan_reduce argument that
// reproduces any rank's; for the ring, elements [0, U) take `p` and [U, count) `rem`, counted from
// U; ranges split over the ranks when every rank's programs agree).  MN_TWO_LEVEL: `node` = the
// node step's programs for local rank 0 over the node's ranks, `lead` = the leaders' programs over
// the nodes' partials for the leader whose result this rank takes (its own node's, or for
// MPI_Reduce the root's node).  big: more ranks (MN_FLAT) or nodes (MN_TWO_LEVEL's leaders) than
// a program holds (kMaxRanks): the host evaluates the message schedule itself (mpi/user_coll.cpp):
// forced ALG_PT2PT_RD = recursive doubling, ALG_RING = the ring over [0, U) and recursive doubling
// on the rest, ALG_BINOMIAL / ALG_KNOMIAL (factor k) / ALG_REDSCAT_GATHER = that reduce to `root` (a
// node index for the leaders).
enum : int { MN_FLAT = 0, MN_TWO_LEVEL = 1 };
enum : int { MN_COLL_ALLREDUCE = 0, MN_COLL_REDUCE = 1 };
struct MnSched {
    int kind;
    int forced;
    long U;
    int coll, big, root, k;  // k: the knomial factor (forced ALG_KNOMIAL)
    Plan p, rem, node, lead;
};
int mn_host_schedule(int coll, size_t count, int tsize, int textent, bool in_place, int opk, int root, MnSched *s);

const char *algo_name(int algo);

}  // namespace mv2
