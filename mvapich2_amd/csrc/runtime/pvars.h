// pvars.h — MPI_T performance variables of the collective hot path: per
// algorithm call counters and timers under the reference's names
// (src/mpi_t/mv2_mpit.c: MPIR_T_PVAR_COUNTER_REGISTER_STATIC /
// MPIR_T_PVAR_TIMER_REGISTER_STATIC, categories "Allreduce Algorithms",
// "Reduce Algorithms", "Reduce_scatter Algorithms", "Shmem Collective Calls").
// A call increments the counters the reference's call chain for the selected
// algorithm increments (its MPIR_T_PVAR_COUNTER_INC sites, cited per entry in
// pvars.cpp) and adds the call's wall time to the matching timers.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "orders.h"

namespace mv2 {

enum PvarId : int {
    PV_AR_SHM_RD, PV_AR_SHM_RS, PV_AR_SHM_INTRA, PV_AR_INTRA_P2P, PV_AR_2LVL, PV_AR_TOPO,
    PV_AR_RING, PV_AR_RING_WRAPPER, PV_AR_RING_INPLACE,
    PV_RED_BINOMIAL, PV_RED_REDSCAT_GATHER, PV_RED_SHMEM, PV_RED_KNOMIAL, PV_RED_TOPO, PV_RED_TWO_LEVEL_HELPER,
    PV_RS_BASIC, PV_RS_REC_HALVING, PV_RS_PAIRWISE, PV_RS_RING, PV_RS_RING_2LVL, PV_RS_NON_COMM, PV_RS_NONCOMM,
    PV_NUM_SHMEM_COLL_CALLS,
    PV_COUNT
};

struct PvarDesc {
    const char *counter;   // MPI_T name of the call counter (MPI_UNSIGNED_LONG_LONG)
    const char *timer;     // MPI_T name of the timer (MPI_DOUBLE seconds), or nullptr
    const char *category;
    const char *desc;
};
const PvarDesc &pvar_desc(int id);
uint64_t pvar_count(int id);
double pvar_seconds(int id);

enum { PV_COLL_ALLREDUCE = 0, PV_COLL_REDUCE = 1, PV_COLL_REDUCE_SCATTER = 2 };

// Bracket one API call: begin/end nest (only the outermost call commits), and
// the first note inside records the selected plan's counter chain.
void pvar_begin();
void pvar_note(int coll, const Plan &p, bool in_place, size_t count, int n);
void pvar_note_id(int id);
void pvar_note_ids(const int *ids, int n);  // a whole chain; later notes in the call are ignored
void pvar_end(bool ok);

}  // namespace mv2
