/* mv2amd_collops.h — the device collectives as MVAPICH2 coll-function-table
 * entries, for a maintainer who keeps MVAPICH2's MPI layer and swaps only the
 * hot path.
 *
 * Replaces, per intracommunicator: the MPID_Collops members (reference
 * src/include/mpiimpl.h:1999-2033) that MPIDI_CH3I_comm_create installs
 * (src/mpid/ch3/channels/mrail/src/rdma/ch3i_comm.c:83-98):
 *   Barrier, Bcast, Allgather, Reduce, Allreduce, Reduce_scatter,
 *   Reduce_scatter_block.
 * Each function has exactly the member's signature; MPID_Comm stays opaque
 * (only its address is used, to find the attachment below).
 *
 * Contract:
 *  - libmpi.so's node world is initialised (mv2h_init, from the launcher's
 *    RANK / MV2_COMM_WORLD_* variables) and the communicator was attached with
 *    MV2AMD_Comm_attach(comm, rank, size), which succeeds only when the
 *    communicator is that world in rank order.  Anything else returns
 *    MPI_ERR_COMM without side effects, so the caller falls back to the
 *    MVAPICH2 function it replaced.
 *  - Builtin datatypes and builtin ops only (handles are MPICH ABI, equal in
 *    both libraries); a derived type or user op returns MPI_ERR_TYPE /
 *    MPI_ERR_OP before any data moves (fall back).
 *  - Buffers may be device (hipMalloc) or host memory; device buffers are the
 *    reason to install this.  MPI_IN_PLACE as in the MPI standard.
 *  - Errors: the MPI error class is returned and *errflag is set to
 *    MPIR_ERR_OTHER (= MPI_ERR_OTHER), like the MV2 algorithms
 *    (mpir_type_defs.h:15-19).  Results are bit-identical to the algorithms
 *    MVAPICH2 2.3.7 would have selected for the same call on one node. */
#ifndef MV2AMD_COLLOPS_H
#define MV2AMD_COLLOPS_H

#include "mpi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct MPID_Comm MPID_Comm; /* MVAPICH2's communicator object: opaque here */
typedef int MPIR_Errflag_t;         /* MPIR_ERR_NONE = 0, MPIR_ERR_OTHER = MPI_ERR_OTHER */

int MV2AMD_Comm_attach(MPID_Comm *comm, int rank, int size);
int MV2AMD_Comm_detach(MPID_Comm *comm);

int MV2AMD_Barrier(MPID_Comm *comm, MPIR_Errflag_t *errflag);
int MV2AMD_Bcast(void *buffer, int count, MPI_Datatype datatype, int root, MPID_Comm *comm, MPIR_Errflag_t *errflag);
int MV2AMD_Allgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf, int recvcount,
                     MPI_Datatype recvtype, MPID_Comm *comm, MPIR_Errflag_t *errflag);
int MV2AMD_Reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op, int root,
                  MPID_Comm *comm, MPIR_Errflag_t *errflag);
int MV2AMD_Allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                     MPID_Comm *comm, MPIR_Errflag_t *errflag);
int MV2AMD_Reduce_scatter(const void *sendbuf, void *recvbuf, const int *recvcnts, MPI_Datatype datatype,
                          MPI_Op op, MPID_Comm *comm, MPIR_Errflag_t *errflag);
int MV2AMD_Reduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount, MPI_Datatype datatype,
                                MPI_Op op, MPID_Comm *comm, MPIR_Errflag_t *errflag);

/* The members above, in MPID_Collops' member order, for copying into a table. */
typedef struct MV2AMD_Collops {
    int (*Barrier)(MPID_Comm *, MPIR_Errflag_t *);
    int (*Bcast)(void *, int, MPI_Datatype, int, MPID_Comm *, MPIR_Errflag_t *);
    int (*Allgather)(const void *, int, MPI_Datatype, void *, int, MPI_Datatype, MPID_Comm *, MPIR_Errflag_t *);
    int (*Reduce)(const void *, void *, int, MPI_Datatype, MPI_Op, int, MPID_Comm *, MPIR_Errflag_t *);
    int (*Allreduce)(const void *, void *, int, MPI_Datatype, MPI_Op, MPID_Comm *, MPIR_Errflag_t *);
    int (*Reduce_scatter)(const void *, void *, const int *, MPI_Datatype, MPI_Op, MPID_Comm *, MPIR_Errflag_t *);
    int (*Reduce_scatter_block)(const void *, void *, int, MPI_Datatype, MPI_Op, MPID_Comm *, MPIR_Errflag_t *);
} MV2AMD_Collops;

int MV2AMD_Collops_get(MV2AMD_Collops *ops);

#ifdef __cplusplus
}
#endif
#endif
