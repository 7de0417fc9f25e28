// pvars.cpp — see pvars.h.
#include "pvars.h"

#include <time.h>

#include <atomic>

namespace mv2 {

namespace {

const PvarDesc kDesc[PV_COUNT] = {
    // MPIR_Allreduce_pt2pt_rd_MV2 allreduce_osu.c:366-367
    {"mv2_coll_allreduce_shm_rd", "mv2_coll_timer_allreduce_shm_rd", "Allreduce Algorithms",
     "Number of times MV2 shm rd allreduce algorithm was invoked"},
    // MPIR_Allreduce_pt2pt_rs_MV2 :639-640
    {"mv2_coll_allreduce_shm_rs", "mv2_coll_timer_allreduce_shm_rs", "Allreduce Algorithms",
     "Number of times MV2 shm rs allreduce algorithm was invoked"},
    // MPIR_Allreduce_reduce_shmem_MV2 :1488-1489
    {"mv2_coll_allreduce_shm_intra", "mv2_coll_timer_allreduce_shm_intra", "Allreduce Algorithms",
     "Number of times MV2 shm intra allreduce algorithm was invoked"},
    // MPIR_Allreduce_reduce_p2p_MV2 :1622-1623
    {"mv2_coll_allreduce_intra_p2p", "mv2_coll_timer_allreduce_intra_p2p", "Allreduce Algorithms",
     "Number of times MV2 intra p2p allreduce algorithm was invoked"},
    // MPIR_Allreduce_two_level_MV2 :1693-1694
    {"mv2_coll_allreduce_2lvl", "mv2_coll_timer_allreduce_2lvl", "Allreduce Algorithms",
     "Number of times MV2 two-level allreduce algorithm was invoked"},
    // MPIR_Allreduce_topo_aware_hierarchical_MV2 :2278-2279
    {"mv2_coll_allreduce_topo_aware_hierarchical", "mv2_coll_timer_allreduce_topo_aware_hierarchical",
     "Allreduce Algorithms", "Number of times MV2 topo-aware hierarchical allreduce algorithm was invoked"},
    // MPIR_Allreduce_pt2pt_ring_MV2 :3898-3899 (after its fallback test :3893)
    {"mv2_coll_allreduce_pt2pt_ring", "mv2_coll_timer_allreduce_pt2pt_ring", "Allreduce Algorithms",
     "Number of times MV2 pt2pt ring allreduce algorithm was invoked"},
    // MPIR_Allreduce_pt2pt_ring_wrapper_MV2 :3761-3762
    {"mv2_coll_allreduce_pt2pt_ring_wrapper", "mv2_coll_timer_allreduce_pt2pt_ring_wrapper", "Allreduce Algorithms",
     "Number of times MV2 pt2pt ring wrapper allreduce algorithm was invoked"},
    // MPIR_Allreduce_pt2pt_ring_inplace_MV2 :4103-4104 (after its fallback test :4095)
    {"mv2_coll_allreduce_pt2pt_ring_inplace", "mv2_coll_timer_allreduce_pt2pt_ring_inplace", "Allreduce Algorithms",
     "Number of times MV2 pt2pt ring in-place allreduce algorithm was invoked"},
    // MPIR_Reduce_binomial_MV2 reduce_osu.c:450
    {"mv2_coll_reduce_binomial", "mv2_coll_timer_reduce_binomial", "Reduce Algorithms",
     "Number of times MV2 binomial reduce algorithm was invoked"},
    // MPIR_Reduce_redscat_gather_MV2 :745
    {"mv2_coll_reduce_redscat_gather", "mv2_coll_timer_reduce_redscat_gather", "Reduce Algorithms",
     "Number of times MV2 redscat-gather reduce algorithm was invoked"},
    // MPIR_Reduce_shmem_MV2 :1187
    {"mv2_coll_reduce_shmem", "mv2_coll_timer_reduce_shmem", "Reduce Algorithms",
     "Number of times MV2 shmem reduce algorithm was invoked"},
    // MPIR_Reduce_knomial_MV2 :1672 (also under MPIR_Reduce_intra_knomial_wrapper_MV2 :1878)
    {"mv2_coll_reduce_knomial", "mv2_coll_timer_reduce_knomial", "Reduce Algorithms",
     "Number of times MV2 knomial reduce algorithm was invoked"},
    // MPIR_Reduce_topo_aware_hierarchical_MV2 :160
    {"mv2_coll_reduce_topo_aware_hierarchical", "mv2_coll_timer_reduce_topo_aware_hierarchical", "Reduce Algorithms",
     "Number of times MV2 topo-aware hierarchical reduce algorithm was invoked"},
    // MPIR_Reduce_two_level_helper_MV2 :2039
    {"mv2_coll_reduce_two_level_helper", "mv2_coll_timer_reduce_two_level_helper", "Reduce Algorithms",
     "Number of times MV2 two-level helper reduce algorithm was invoked"},
    // MPIR_Reduce_Scatter_Basic_MV2 red_scat_osu.c:317
    {"mv2_coll_reduce_scatter_basic", "mv2_coll_timer_reduce_scatter_basic", "Reduce_scatter Algorithms",
     "Number of times MV2 basic reduce_scatter algorithm was invoked"},
    // MPIR_Reduce_scatter_Rec_Halving_MV2 :456
    {"mv2_coll_reduce_scatter_rec_halving", "mv2_coll_timer_reduce_scatter_rec_halving", "Reduce_scatter Algorithms",
     "Number of times MV2 recursive-halving reduce_scatter algorithm was invoked"},
    // MPIR_Reduce_scatter_Pair_Wise_MV2 :810
    {"mv2_coll_reduce_scatter_pairwise", "mv2_coll_timer_reduce_scatter_pairwise", "Reduce_scatter Algorithms",
     "Number of times MV2 pairwise reduce_scatter algorithm was invoked"},
    // MPIR_Reduce_scatter_ring :1039 (MPIR_Reduce_scatter_ring_2lvl hands over to it while the
    // communicator has no rank_list, :1200-1205)
    {"mv2_coll_reduce_scatter_ring", "mv2_coll_timer_reduce_scatter_ring", "Reduce_scatter Algorithms",
     "Number of times MV2 ring reduce_scatter algorithm was invoked"},
    // MPIR_Reduce_scatter_ring_2lvl :1209: only once MVAPICH2 has built an allgather
    // communicator (create_allgather_comm, create_2level_comm.c:1523), never on this path
    {"mv2_coll_reduce_scatter_ring_2lvl", "mv2_coll_timer_reduce_scatter_ring_2lvl", "Reduce_scatter Algorithms",
     "Number of times MV2 two-level ring reduce_scatter algorithm was invoked"},
    // MPIR_Reduce_scatter_non_comm_MV2 :1394
    {"mv2_coll_reduce_scatter_non_comm", "mv2_coll_timer_reduce_scatter_non_comm", "Reduce_scatter Algorithms",
     "Number of times MV2 non-commutative reduce_scatter algorithm was invoked"},
    // MPIR_Reduce_scatter_noncomm_MV2 :154 (pof2 size, equal counts, inside the above)
    {"mv2_coll_reduce_scatter_noncomm", "mv2_coll_timer_reduce_scatter_noncomm", "Reduce_scatter Algorithms",
     "Number of times MV2 power-of-two non-commutative reduce_scatter algorithm was invoked"},
    // reduce_shmem (allreduce_osu.c:1513) and MPIR_Reduce_shmem_MV2's shmem slot use
    {"mv2_num_shmem_coll_calls", nullptr, "Shmem Collective Calls",
     "Number of times MV2 shared-memory collective calls were invoked"},
};

std::atomic<uint64_t> g_count[PV_COUNT];
std::atomic<uint64_t> g_ns[PV_COUNT];

struct CallRec {
    int depth = 0;
    bool noted = false;
    int n = 0;
    int ids[16];
    uint64_t t0 = 0;
};
thread_local CallRec t_rec;

uint64_t now_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

void push(int id) {
    if (t_rec.n < 16) t_rec.ids[t_rec.n++] = id;
}

// MPIR_Reduce_MV2's chain for a reduce plan
void reduce_chain(const Plan &p, int algo) {
    if (p.via & VIA_TWO_LEVEL_HELPER) push(PV_RED_TWO_LEVEL_HELPER);
    switch (algo) {
    case ALG_SHMEM_LINEAR: push(PV_RED_SHMEM); push(PV_NUM_SHMEM_COLL_CALLS); break;
    case ALG_KNOMIAL: push(PV_RED_KNOMIAL); break;
    case ALG_BINOMIAL: push(PV_RED_BINOMIAL); break;
    case ALG_REDSCAT_GATHER: push(PV_RED_REDSCAT_GATHER); break;
    case ALG_REDUCE_TOPO: push(PV_RED_TOPO); break;
    default: break;
    }
}

}  // namespace

const PvarDesc &pvar_desc(int id) { return kDesc[id]; }
uint64_t pvar_count(int id) { return g_count[id].load(std::memory_order_relaxed); }
double pvar_seconds(int id) { return 1e-9 * (double)g_ns[id].load(std::memory_order_relaxed); }

void pvar_begin() {
    if (t_rec.depth++ == 0) {
        t_rec.noted = false;
        t_rec.n = 0;
        t_rec.t0 = now_ns();
    }
}

void pvar_note_id(int id) {
    if (t_rec.depth != 1 || t_rec.noted || nbc_kind() != NBC_NONE) return;
    t_rec.noted = true;
    push(id);
}

void pvar_note_ids(const int *ids, int n) {
    if (t_rec.depth != 1 || t_rec.noted || nbc_kind() != NBC_NONE) return;
    t_rec.noted = true;
    for (int i = 0; i < n; ++i) push(ids[i]);
}

void pvar_note(int coll, const Plan &p, bool in_place, size_t count, int n) {
    // nonblocking initiations run the MPI_I* schedules, whose mv2_coll_i* counters are not
    // among these variables
    if (t_rec.depth != 1 || t_rec.noted || p.algo == ALG_NONE || nbc_kind() != NBC_NONE) return;
    t_rec.noted = true;
    switch (coll) {
    case PV_COLL_ALLREDUCE:
        switch (p.algo) {
        case ALG_TOPO_TREE: push(PV_AR_TOPO); break;
        case ALG_SHMEM_LINEAR:  // two-level with reduce_shmem (:1693, :1488, :1513)
            push(PV_AR_2LVL); push(PV_AR_SHM_INTRA); push(PV_NUM_SHMEM_COLL_CALLS);
            break;
        case ALG_TWO_LEVEL_P2P:  // two-level with reduce_p2p -> MPIR_Reduce_MV2 (:1622)
            push(PV_AR_2LVL); push(PV_AR_INTRA_P2P);
            reduce_chain(p, p.inner);
            break;
        case ALG_PT2PT_RS: push(PV_AR_SHM_RS); break;
        case ALG_PT2PT_RD: push((p.via & VIA_RS_ENTRY) ? PV_AR_SHM_RS : PV_AR_SHM_RD); break;
        case ALG_RING: {
            // wrapper (:3761); the ring body over (count/n)*n elements runs unless it falls back
            // to pt2pt_rs (count < n or IN_PLACE, :3893 / :4095); the remainder is pt2pt_rs (:3800)
            push(PV_AR_RING_WRAPPER);
            push(count >= (size_t)n && !in_place ? PV_AR_RING : PV_AR_SHM_RS);
            if (count % (size_t)n) push(PV_AR_SHM_RS);
            break;
        }
        default: break;
        }
        break;
    case PV_COLL_REDUCE: reduce_chain(p, p.algo); break;
    case PV_COLL_REDUCE_SCATTER:
        switch (p.algo) {
        case ALG_RS_RING: push(PV_RS_RING); break;
        case ALG_RS_REC_HALVING: push(PV_RS_REC_HALVING); break;
        case ALG_RS_PAIRWISE: push(PV_RS_PAIRWISE); break;
        case ALG_RS_BASIC: push(PV_RS_BASIC); reduce_chain(p, p.inner); break;
        case ALG_RS_NONCOMM_POF2: push(PV_RS_NON_COMM); push(PV_RS_NONCOMM); break;
        case ALG_RS_NONCOMM_RD: push(PV_RS_NON_COMM); break;
        default: break;
        }
        break;
    default: break;
    }
}

void pvar_end(bool ok) {
    if (t_rec.depth <= 0) return;
    if (--t_rec.depth) return;
    if (!ok) return;
    const uint64_t dt = now_ns() - t_rec.t0;
    for (int i = 0; i < t_rec.n; ++i) {
        g_count[t_rec.ids[i]].fetch_add(1, std::memory_order_relaxed);
        g_ns[t_rec.ids[i]].fetch_add(dt, std::memory_order_relaxed);
    }
}

}  // namespace mv2
