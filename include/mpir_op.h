/* mpir_op.h — the predefined MPI_Op functions of libmpi.so as
 * MPI_User_function entry points, for code that calls the op layer directly
 * the way MVAPICH2's collectives do (MPIR_OP_HDL_TO_FN(op)(in, inout, &len,
 * &type)).
 *
 * Replaces: MPIR_Op_table / MPIR_Op_check_dtype_table (reference
 * src/mpi/coll/allreduce.c:95-107, declared src/include/mpiimpl.h:4010-4032)
 * and the per-op functions MPIR_SUM ... MPIR_NO_OP (src/mpi/coll/op*.c).
 *
 * Difference from the reference: the buffers may be device memory (hipMalloc);
 * the op then runs as one gfx950 kernel and returns when inoutvec holds the
 * result.  Host buffers are accepted too (staged through the GPU; x87 long
 * double types are reduced on the host).  A type the op does not accept
 * leaves inoutvec untouched and records MPI_ERR_OP, read (and cleared) with
 * MPIR_Op_errno() — the reference keeps it in the thread-private op_errno. */
#ifndef MV2AMD_MPIR_OP_H
#define MV2AMD_MPIR_OP_H

#include "mpi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef int(MPIR_Op_check_dtype_fn)(MPI_Datatype);

#define MPIR_PREDEF_OP_COUNT 14
extern MPI_User_function *MPIR_Op_table[];
extern MPIR_Op_check_dtype_fn *MPIR_Op_check_dtype_table[];
#define MPIR_OP_HDL_TO_FN(op) MPIR_Op_table[((op)&0xf) - 1]
#define MPIR_OP_HDL_TO_DTYPE_FN(op) MPIR_Op_check_dtype_table[((op)&0xf) - 1]

void MPIR_MAXF(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_MINF(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_SUM(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_PROD(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_LAND(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_BAND(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_LOR(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_BOR(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_LXOR(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_BXOR(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_MINLOC(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_MAXLOC(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_REPLACE(void *invec, void *inoutvec, int *len, MPI_Datatype *type);
void MPIR_NO_OP(void *invec, void *inoutvec, int *len, MPI_Datatype *type);

int MPIR_MAXF_check_dtype(MPI_Datatype type);
int MPIR_MINF_check_dtype(MPI_Datatype type);
int MPIR_SUM_check_dtype(MPI_Datatype type);
int MPIR_PROD_check_dtype(MPI_Datatype type);
int MPIR_LAND_check_dtype(MPI_Datatype type);
int MPIR_BAND_check_dtype(MPI_Datatype type);
int MPIR_LOR_check_dtype(MPI_Datatype type);
int MPIR_BOR_check_dtype(MPI_Datatype type);
int MPIR_LXOR_check_dtype(MPI_Datatype type);
int MPIR_BXOR_check_dtype(MPI_Datatype type);
int MPIR_MINLOC_check_dtype(MPI_Datatype type);
int MPIR_MAXLOC_check_dtype(MPI_Datatype type);
int MPIR_REPLACE_check_dtype(MPI_Datatype type);
int MPIR_NO_OP_check_dtype(MPI_Datatype type);

/* the error of the last op call on this thread (MPI_SUCCESS if none); clears it */
int MPIR_Op_errno(void);

#ifdef __cplusplus
}
#endif
#endif
