// collops.cpp — include/mv2amd_collops.h: the device collectives behind
// MVAPICH2's coll function table (MPID_Collops, mpiimpl.h:1999-2033).  The
// MVAPICH2 MPI layer has already checked the arguments (e.g. allreduce.c:
// 827-960), so these go straight to the C-ABI; anything this path does not
// cover returns an error before data moves so the caller can fall back.
#include <stddef.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "../../../include/mpi.h"
#include "../../../include/mv2amd_collops.h"
#include "../../../include/mv2h.h"

namespace {

std::mutex g_mu;
std::vector<MPID_Comm *> g_attached;

bool attached(MPID_Comm *c) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (MPID_Comm *a : g_attached)
        if (a == c) return true;
    return false;
}

// MPI class -> (class, *errflag) as the MV2 algorithms report it
int fail(int rc, MPIR_Errflag_t *errflag) {
    if (rc && errflag) *errflag = MPI_ERR_OTHER;
    return rc;
}

// builtin type + builtin op this path reduces on the device
int check_reduce(MPI_Datatype dt, MPI_Op op, size_t *ext) {
    size_t size = 0;
    if (mv2h_dtype_info(dt, &size, ext)) return MPI_ERR_TYPE;
    return mv2h_op_check(op, dt) ? MPI_ERR_OP : MPI_SUCCESS;
}

}  // namespace

extern "C" {

int MV2AMD_Comm_attach(MPID_Comm *comm, int rank, int size) {
    if (!comm || rank != mv2h_rank() || size != mv2h_size()) return MPI_ERR_COMM;
    std::lock_guard<std::mutex> lk(g_mu);
    for (MPID_Comm *a : g_attached)
        if (a == comm) return MPI_SUCCESS;
    g_attached.push_back(comm);
    return MPI_SUCCESS;
}

int MV2AMD_Comm_detach(MPID_Comm *comm) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (size_t i = 0; i < g_attached.size(); ++i)
        if (g_attached[i] == comm) {
            g_attached.erase(g_attached.begin() + i);
            return MPI_SUCCESS;
        }
    return MPI_ERR_COMM;
}

int MV2AMD_Barrier(MPID_Comm *comm, MPIR_Errflag_t *errflag) {
    if (!attached(comm)) return MPI_ERR_COMM;
    return fail(mv2h_barrier(), errflag);
}

int MV2AMD_Bcast(void *buffer, int count, MPI_Datatype dt, int root, MPID_Comm *comm, MPIR_Errflag_t *errflag) {
    if (!attached(comm)) return MPI_ERR_COMM;
    size_t size = 0, ext = 0;
    if (mv2h_dtype_info(dt, &size, &ext)) return MPI_ERR_TYPE;
    if (count == 0) return MPI_SUCCESS;
    return fail(mv2h_bcast(buffer, (size_t)count * ext, root, nullptr), errflag);
}

int MV2AMD_Allgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf, int recvcount,
                     MPI_Datatype recvtype, MPID_Comm *comm, MPIR_Errflag_t *errflag) {
    if (!attached(comm)) return MPI_ERR_COMM;
    size_t rs = 0, rext = 0;
    if (mv2h_dtype_info(recvtype, &rs, &rext)) return MPI_ERR_TYPE;
    const size_t rbytes = (size_t)recvcount * rext;
    if (sendbuf != MPI_IN_PLACE) {
        size_t ss = 0, sext = 0;
        if (mv2h_dtype_info(sendtype, &ss, &sext)) return MPI_ERR_TYPE;
        if ((size_t)sendcount * sext != rbytes) return MPI_ERR_TRUNCATE;
    }
    if (rbytes == 0) return MPI_SUCCESS;
    return fail(mv2h_allgather(sendbuf, recvbuf, rbytes, nullptr), errflag);
}

int MV2AMD_Reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, int root,
                  MPID_Comm *comm, MPIR_Errflag_t *errflag) {
    if (!attached(comm)) return MPI_ERR_COMM;
    size_t ext = 0;
    if (int rc = check_reduce(dt, op, &ext)) return rc;
    if (count == 0) return MPI_SUCCESS;
    return fail(mv2h_reduce(sendbuf, recvbuf, (size_t)count, dt, op, root, nullptr), errflag);
}

int MV2AMD_Allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, MPID_Comm *comm,
                     MPIR_Errflag_t *errflag) {
    if (!attached(comm)) return MPI_ERR_COMM;
    size_t ext = 0;
    if (int rc = check_reduce(dt, op, &ext)) return rc;
    if (count == 0) return MPI_SUCCESS;
    return fail(mv2h_allreduce(sendbuf, recvbuf, (size_t)count, dt, op, nullptr), errflag);
}

int MV2AMD_Reduce_scatter(const void *sendbuf, void *recvbuf, const int *recvcnts, MPI_Datatype dt, MPI_Op op,
                          MPID_Comm *comm, MPIR_Errflag_t *errflag) {
    if (!attached(comm)) return MPI_ERR_COMM;
    size_t ext = 0;
    if (int rc = check_reduce(dt, op, &ext)) return rc;
    const int n = mv2h_size();
    std::vector<size_t> counts((size_t)n);
    for (int j = 0; j < n; ++j) {
        if (recvcnts[j] < 0) return MPI_ERR_COUNT;
        counts[(size_t)j] = (size_t)recvcnts[j];
    }
    return fail(mv2h_reduce_scatter(sendbuf, recvbuf, counts.data(), dt, op, nullptr), errflag);
}

int MV2AMD_Reduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount, MPI_Datatype dt, MPI_Op op,
                                MPID_Comm *comm, MPIR_Errflag_t *errflag) {
    if (!attached(comm)) return MPI_ERR_COMM;
    size_t ext = 0;
    if (int rc = check_reduce(dt, op, &ext)) return rc;
    if (recvcount < 0) return MPI_ERR_COUNT;
    std::vector<size_t> counts((size_t)mv2h_size(), (size_t)recvcount);
    // MPIR_Reduce_scatter_block_MV2 runs MPICH's reduce_scatter_block selection (see
    // PMPI_Reduce_scatter_block, mpi_api.cpp)
    mv2h_nbc_begin(MV2H_NBC_IREDUCE_SCATTER_BLOCK);
    const int rc = mv2h_reduce_scatter(sendbuf, recvbuf, counts.data(), dt, op, nullptr);
    mv2h_nbc_end();
    return fail(rc, errflag);
}

int MV2AMD_Collops_get(MV2AMD_Collops *ops) {
    if (!ops) return MPI_ERR_ARG;
    ops->Barrier = MV2AMD_Barrier;
    ops->Bcast = MV2AMD_Bcast;
    ops->Allgather = MV2AMD_Allgather;
    ops->Reduce = MV2AMD_Reduce;
    ops->Allreduce = MV2AMD_Allreduce;
    ops->Reduce_scatter = MV2AMD_Reduce_scatter;
    ops->Reduce_scatter_block = MV2AMD_Reduce_scatter_block;
    return MPI_SUCCESS;
}

}  // extern "C"
