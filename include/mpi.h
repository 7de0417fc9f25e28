/*
 * mpi.h — MPI-3.1 C API subset exported by libmpi.so (mvapich2_amd).
 *
 * Drop-in boundary for the device-buffer reduction / collective hot path of
 * MVAPICH2 2.3.7.  Handle values follow the MPICH ABI of the reference build
 * (LP64, x86-64) so object code compiled against the reference's mpi.h calls
 * into this library unchanged:
 *   - datatype encodings   reference configure.ac:3475-3530, 3707-3733
 *   - op handles           reference src/include/mpi.h.in:314-327
 *   - comm handles         reference src/include/mpi.h.in:292-293
 *   - error classes        reference src/include/mpi.h.in:796-865
 *   - MPI_IN_PLACE         reference src/include/mpi.h.in:557
 * Every MPI_X symbol is a weak alias of PMPI_X (reference allreduce.c:80-84).
 *
 * Buffers passed to the collective entry points may be device (hipMalloc)
 * pointers; that is the path this library implements on MI355X.
 */
#ifndef MV2AMD_MPI_H_INCLUDED
#define MV2AMD_MPI_H_INCLUDED

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int MPI_Datatype;
typedef int MPI_Op;
typedef int MPI_Comm;
typedef int MPI_Errhandler;
typedef int MPI_Group;
typedef int MPI_Request;
typedef long MPI_Aint;
typedef long long MPI_Offset;
typedef long long MPI_Count;
typedef int MPI_Fint;

typedef struct MPI_Status {
    int count_lo;
    int count_hi_and_cancelled;
    int MPI_SOURCE;
    int MPI_TAG;
    int MPI_ERROR;
} MPI_Status;

typedef void(MPI_User_function)(void *, void *, int *, MPI_Datatype *);

/* ---- null handles / special values ---- */
#define MPI_DATATYPE_NULL ((MPI_Datatype)0x0c000000)
#define MPI_OP_NULL ((MPI_Op)0x18000000)
#define MPI_COMM_NULL ((MPI_Comm)0x04000000)
#define MPI_COMM_WORLD ((MPI_Comm)0x44000000)
#define MPI_COMM_SELF ((MPI_Comm)0x44000001)
#define MPI_ERRHANDLER_NULL ((MPI_Errhandler)0x14000000)
#define MPI_ERRORS_ARE_FATAL ((MPI_Errhandler)0x54000000)
#define MPI_ERRORS_RETURN ((MPI_Errhandler)0x54000001)
#define MPI_IN_PLACE ((void *)-1)
#define MPI_BOTTOM ((void *)0)
#define MPI_UNDEFINED (-32766)
#define MPI_STATUS_IGNORE ((MPI_Status *)1)
#define MPI_STATUSES_IGNORE ((MPI_Status *)1)
#define MPI_REQUEST_NULL ((MPI_Request)0x2c000000)
#define MPI_ANY_SOURCE (-2)
#define MPI_ANY_TAG (-1)
#define MPI_PROC_NULL (-1)
#define MPI_TAG_UB_VALUE 0x7fffffff
#define MPI_MAX_PROCESSOR_NAME 128
#define MPI_MAX_ERROR_STRING 512
#define MPI_MAX_OBJECT_NAME 128
#define MPI_THREAD_SINGLE 0
#define MPI_THREAD_FUNNELED 1
#define MPI_THREAD_SERIALIZED 2
#define MPI_THREAD_MULTIPLE 3
#define MPI_VERSION 3
#define MPI_SUBVERSION 1

/* ---- predefined datatypes (MPICH ABI, LP64) ---- */
#define MPI_CHAR ((MPI_Datatype)0x4c000101)
#define MPI_SIGNED_CHAR ((MPI_Datatype)0x4c000118)
#define MPI_UNSIGNED_CHAR ((MPI_Datatype)0x4c000102)
#define MPI_BYTE ((MPI_Datatype)0x4c00010d)
#define MPI_WCHAR ((MPI_Datatype)0x4c00040e)
#define MPI_SHORT ((MPI_Datatype)0x4c000203)
#define MPI_UNSIGNED_SHORT ((MPI_Datatype)0x4c000204)
#define MPI_INT ((MPI_Datatype)0x4c000405)
#define MPI_UNSIGNED ((MPI_Datatype)0x4c000406)
#define MPI_LONG ((MPI_Datatype)0x4c000807)
#define MPI_UNSIGNED_LONG ((MPI_Datatype)0x4c000808)
#define MPI_FLOAT ((MPI_Datatype)0x4c00040a)
#define MPI_DOUBLE ((MPI_Datatype)0x4c00080b)
#define MPI_LONG_DOUBLE ((MPI_Datatype)0x4c00100c)
#define MPI_LONG_LONG_INT ((MPI_Datatype)0x4c000809)
#define MPI_LONG_LONG MPI_LONG_LONG_INT
#define MPI_UNSIGNED_LONG_LONG ((MPI_Datatype)0x4c000819)
#define MPI_PACKED ((MPI_Datatype)0x4c00010f)
#define MPI_LB ((MPI_Datatype)0x4c000010)
#define MPI_UB ((MPI_Datatype)0x4c000011)
#define MPI_FLOAT_INT ((MPI_Datatype)0x8c000000)
#define MPI_DOUBLE_INT ((MPI_Datatype)0x8c000001)
#define MPI_LONG_INT ((MPI_Datatype)0x8c000002)
#define MPI_SHORT_INT ((MPI_Datatype)0x8c000003)
#define MPI_2INT ((MPI_Datatype)0x4c000816)
#define MPI_LONG_DOUBLE_INT ((MPI_Datatype)0x8c000004)
#define MPI_INT8_T ((MPI_Datatype)0x4c000137)
#define MPI_INT16_T ((MPI_Datatype)0x4c000238)
#define MPI_INT32_T ((MPI_Datatype)0x4c000439)
#define MPI_INT64_T ((MPI_Datatype)0x4c00083a)
#define MPI_UINT8_T ((MPI_Datatype)0x4c00013b)
#define MPI_UINT16_T ((MPI_Datatype)0x4c00023c)
#define MPI_UINT32_T ((MPI_Datatype)0x4c00043d)
#define MPI_UINT64_T ((MPI_Datatype)0x4c00083e)
#define MPI_C_BOOL ((MPI_Datatype)0x4c00013f)
#define MPI_C_FLOAT_COMPLEX ((MPI_Datatype)0x4c000840)
#define MPI_C_COMPLEX MPI_C_FLOAT_COMPLEX
#define MPI_C_DOUBLE_COMPLEX ((MPI_Datatype)0x4c001041)
#define MPI_C_LONG_DOUBLE_COMPLEX ((MPI_Datatype)0x4c002042)
#define MPI_AINT ((MPI_Datatype)0x4c000843)
#define MPI_OFFSET ((MPI_Datatype)0x4c000844)
#define MPI_COUNT ((MPI_Datatype)0x4c000845)
/* Fortran types with the gfortran default sizes (configure.ac:3878-4022) */
#define MPI_INTEGER ((MPI_Datatype)0x4c00041b)
#define MPI_REAL ((MPI_Datatype)0x4c00041c)
#define MPI_LOGICAL ((MPI_Datatype)0x4c00041d)
#define MPI_COMPLEX ((MPI_Datatype)0x4c00081e)
#define MPI_DOUBLE_PRECISION ((MPI_Datatype)0x4c00081f)
#define MPI_2INTEGER ((MPI_Datatype)0x4c000820)
#define MPI_2REAL ((MPI_Datatype)0x4c000821)
#define MPI_DOUBLE_COMPLEX ((MPI_Datatype)0x4c001022)
#define MPI_2DOUBLE_PRECISION ((MPI_Datatype)0x4c001023)

/* ---- predefined reduction operations ---- */
#define MPI_MAX ((MPI_Op)0x58000001)
#define MPI_MIN ((MPI_Op)0x58000002)
#define MPI_SUM ((MPI_Op)0x58000003)
#define MPI_PROD ((MPI_Op)0x58000004)
#define MPI_LAND ((MPI_Op)0x58000005)
#define MPI_BAND ((MPI_Op)0x58000006)
#define MPI_LOR ((MPI_Op)0x58000007)
#define MPI_BOR ((MPI_Op)0x58000008)
#define MPI_LXOR ((MPI_Op)0x58000009)
#define MPI_BXOR ((MPI_Op)0x5800000a)
#define MPI_MINLOC ((MPI_Op)0x5800000b)
#define MPI_MAXLOC ((MPI_Op)0x5800000c)
#define MPI_REPLACE ((MPI_Op)0x5800000d)
#define MPI_NO_OP ((MPI_Op)0x5800000e)

/* ---- array orders (MPICH values, mpi.h.in) ---- */
#define MPI_ORDER_C 56
#define MPI_ORDER_FORTRAN 57

/* ---- error classes ---- */
#define MPI_SUCCESS 0
#define MPI_ERR_BUFFER 1
#define MPI_ERR_COUNT 2
#define MPI_ERR_TYPE 3
#define MPI_ERR_TAG 4
#define MPI_ERR_COMM 5
#define MPI_ERR_RANK 6
#define MPI_ERR_ROOT 7
#define MPI_ERR_GROUP 8
#define MPI_ERR_OP 9
#define MPI_ERR_TOPOLOGY 10
#define MPI_ERR_DIMS 11
#define MPI_ERR_ARG 12
#define MPI_ERR_UNKNOWN 13
#define MPI_ERR_TRUNCATE 14
#define MPI_ERR_OTHER 15
#define MPI_ERR_INTERN 16
#define MPI_ERR_IN_STATUS 17
#define MPI_ERR_PENDING 18
#define MPI_ERR_REQUEST 19
#define MPI_ERR_NO_MEM 34
#define MPI_ERR_UNSUPPORTED_OPERATION 44
#define MPI_ERR_LASTCODE 0x3fffffff


/* ---- MPI_T tool information interface (MPICH encodings, mpi.h.in:605-700, :874-892) ---- */
typedef struct MPIR_T_enum_s *MPI_T_enum;
typedef struct MPIR_T_cvar_handle_s *MPI_T_cvar_handle;
typedef struct MPIR_T_pvar_handle_s *MPI_T_pvar_handle;
typedef struct MPIR_T_pvar_session_s *MPI_T_pvar_session;
extern struct MPIR_T_pvar_handle_s *const MPI_T_PVAR_ALL_HANDLES;
#define MPI_T_ENUM_NULL ((MPI_T_enum)0)
#define MPI_T_CVAR_HANDLE_NULL ((MPI_T_cvar_handle)0)
#define MPI_T_PVAR_HANDLE_NULL ((MPI_T_pvar_handle)0)
#define MPI_T_PVAR_SESSION_NULL ((MPI_T_pvar_session)0)
enum MPIR_T_verbosity_t {
    MPI_T_VERBOSITY_USER_BASIC = 221, MPI_T_VERBOSITY_USER_DETAIL, MPI_T_VERBOSITY_USER_ALL,
    MPI_T_VERBOSITY_TUNER_BASIC, MPI_T_VERBOSITY_TUNER_DETAIL, MPI_T_VERBOSITY_TUNER_ALL,
    MPI_T_VERBOSITY_MPIDEV_BASIC, MPI_T_VERBOSITY_MPIDEV_DETAIL, MPI_T_VERBOSITY_MPIDEV_ALL
};
enum MPIR_T_bind_t {
    MPI_T_BIND_NO_OBJECT = 9700, MPI_T_BIND_MPI_COMM, MPI_T_BIND_MPI_DATATYPE, MPI_T_BIND_MPI_ERRHANDLER,
    MPI_T_BIND_MPI_FILE, MPI_T_BIND_MPI_GROUP, MPI_T_BIND_MPI_OP, MPI_T_BIND_MPI_REQUEST, MPI_T_BIND_MPI_WIN,
    MPI_T_BIND_MPI_MESSAGE, MPI_T_BIND_MPI_INFO
};
enum MPIR_T_scope_t {
    MPI_T_SCOPE_CONSTANT = 60438, MPI_T_SCOPE_READONLY, MPI_T_SCOPE_LOCAL, MPI_T_SCOPE_GROUP,
    MPI_T_SCOPE_GROUP_EQ, MPI_T_SCOPE_ALL, MPI_T_SCOPE_ALL_EQ
};
enum MPIR_T_pvar_class_t {
    MPI_T_PVAR_CLASS_STATE = 240, MPI_T_PVAR_CLASS_LEVEL, MPI_T_PVAR_CLASS_SIZE, MPI_T_PVAR_CLASS_PERCENTAGE,
    MPI_T_PVAR_CLASS_HIGHWATERMARK, MPI_T_PVAR_CLASS_LOWWATERMARK, MPI_T_PVAR_CLASS_COUNTER,
    MPI_T_PVAR_CLASS_AGGREGATE, MPI_T_PVAR_CLASS_TIMER, MPI_T_PVAR_CLASS_GENERIC
};
#define MPI_T_ERR_MEMORY 59
#define MPI_T_ERR_NOT_INITIALIZED 60
#define MPI_T_ERR_CANNOT_INIT 61
#define MPI_T_ERR_INVALID_INDEX 62
#define MPI_T_ERR_INVALID_ITEM 63
#define MPI_T_ERR_INVALID_HANDLE 64
#define MPI_T_ERR_OUT_OF_HANDLES 65
#define MPI_T_ERR_OUT_OF_SESSIONS 66
#define MPI_T_ERR_INVALID_SESSION 67
#define MPI_T_ERR_CVAR_SET_NOT_NOW 68
#define MPI_T_ERR_CVAR_SET_NEVER 69
#define MPI_T_ERR_PVAR_NO_STARTSTOP 70
#define MPI_T_ERR_PVAR_NO_WRITE 71
#define MPI_T_ERR_PVAR_NO_ATOMIC 72
#define MPI_T_ERR_INVALID_NAME 73
#define MPI_T_ERR_INVALID 74

/* ---- environment ---- */
int MPI_T_init_thread(int required, int *provided);
int MPI_T_finalize(void);
int MPI_T_enum_get_info(MPI_T_enum enumtype, int *num, char *name, int *name_len);
int MPI_T_enum_get_item(MPI_T_enum enumtype, int indx, int *value, char *name, int *name_len);
int MPI_T_cvar_get_num(int *num_cvar);
int MPI_T_cvar_get_info(int cvar_index, char *name, int *name_len, int *verbosity, MPI_Datatype *datatype,
                        MPI_T_enum *enumtype, char *desc, int *desc_len, int *binding, int *scope);
int MPI_T_cvar_get_index(const char *name, int *cvar_index);
int MPI_T_cvar_handle_alloc(int cvar_index, void *obj_handle, MPI_T_cvar_handle *handle, int *count);
int MPI_T_cvar_handle_free(MPI_T_cvar_handle *handle);
int MPI_T_cvar_read(MPI_T_cvar_handle handle, void *buf);
int MPI_T_cvar_write(MPI_T_cvar_handle handle, const void *buf);
int MPI_T_pvar_get_num(int *num_pvar);
int MPI_T_pvar_get_info(int pvar_index, char *name, int *name_len, int *verbosity, int *var_class,
                        MPI_Datatype *datatype, MPI_T_enum *enumtype, char *desc, int *desc_len, int *binding,
                        int *readonly, int *continuous, int *atomic);
int MPI_T_pvar_get_index(const char *name, int var_class, int *pvar_index);
int MPI_T_pvar_session_create(MPI_T_pvar_session *session);
int MPI_T_pvar_session_free(MPI_T_pvar_session *session);
int MPI_T_pvar_handle_alloc(MPI_T_pvar_session session, int pvar_index, void *obj_handle, MPI_T_pvar_handle *handle,
                            int *count);
int MPI_T_pvar_handle_free(MPI_T_pvar_session session, MPI_T_pvar_handle *handle);
int MPI_T_pvar_start(MPI_T_pvar_session session, MPI_T_pvar_handle handle);
int MPI_T_pvar_stop(MPI_T_pvar_session session, MPI_T_pvar_handle handle);
int MPI_T_pvar_read(MPI_T_pvar_session session, MPI_T_pvar_handle handle, void *buf);
int MPI_T_pvar_write(MPI_T_pvar_session session, MPI_T_pvar_handle handle, const void *buf);
int MPI_T_pvar_reset(MPI_T_pvar_session session, MPI_T_pvar_handle handle);
int MPI_T_pvar_readreset(MPI_T_pvar_session session, MPI_T_pvar_handle handle, void *buf);
int MPI_T_category_get_num(int *num_cat);
int MPI_T_category_get_info(int cat_index, char *name, int *name_len, char *desc, int *desc_len, int *num_cvars,
                            int *num_pvars, int *num_categories);
int MPI_T_category_get_index(const char *name, int *cat_index);
int MPI_T_category_get_cvars(int cat_index, int len, int indices[]);
int MPI_T_category_get_pvars(int cat_index, int len, int indices[]);
int MPI_T_category_get_categories(int cat_index, int len, int indices[]);
int MPI_T_category_changed(int *stamp);

int MPI_Init(int *argc, char ***argv);
int MPI_Init_thread(int *argc, char ***argv, int required, int *provided);
int MPI_Finalize(void);
int MPI_Initialized(int *flag);
int MPI_Finalized(int *flag);
int MPI_Abort(MPI_Comm comm, int errorcode);
double MPI_Wtime(void);
double MPI_Wtick(void);
int MPI_Get_processor_name(char *name, int *resultlen);
int MPI_Error_string(int errorcode, char *string, int *resultlen);
int MPI_Error_class(int errorcode, int *errorclass);
int MPI_Comm_set_errhandler(MPI_Comm comm, MPI_Errhandler errhandler);
int MPI_Comm_get_errhandler(MPI_Comm comm, MPI_Errhandler *errhandler);
int MPI_Errhandler_set(MPI_Comm comm, MPI_Errhandler errhandler);

/* ---- communicators ---- */
int MPI_Comm_rank(MPI_Comm comm, int *rank);
int MPI_Comm_size(MPI_Comm comm, int *size);
int MPI_Barrier(MPI_Comm comm);

/* ---- the hot path: reductions and collectives ---- */
int MPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype,
                     MPI_Op op);
int MPI_Allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                  MPI_Op op, MPI_Comm comm);
int MPI_Reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
               int root, MPI_Comm comm);
int MPI_Reduce_scatter(const void *sendbuf, void *recvbuf, const int recvcounts[],
                       MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
int MPI_Reduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount,
                             MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
int MPI_Allgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf,
                  int recvcount, MPI_Datatype recvtype, MPI_Comm comm);
int MPI_Bcast(void *buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm);

/* ---- nonblocking collectives + request completion (MPI-3.1 5.12, 3.7.3) ---- */
int MPI_Iallreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                   MPI_Op op, MPI_Comm comm, MPI_Request *request);
int MPI_Ireduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                int root, MPI_Comm comm, MPI_Request *request);
int MPI_Ireduce_scatter(const void *sendbuf, void *recvbuf, const int recvcounts[],
                        MPI_Datatype datatype, MPI_Op op, MPI_Comm comm, MPI_Request *request);
int MPI_Ireduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount,
                              MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                              MPI_Request *request);
int MPI_Iallgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf,
                   int recvcount, MPI_Datatype recvtype, MPI_Comm comm, MPI_Request *request);
int MPI_Ibcast(void *buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm,
               MPI_Request *request);
int MPI_Ibarrier(MPI_Comm comm, MPI_Request *request);
int MPI_Wait(MPI_Request *request, MPI_Status *status);
int MPI_Test(MPI_Request *request, int *flag, MPI_Status *status);
int MPI_Waitall(int count, MPI_Request requests[], MPI_Status statuses[]);
int MPI_Testall(int count, MPI_Request requests[], int *flag, MPI_Status statuses[]);
int MPI_Request_free(MPI_Request *request);

/* ---- stream-ordered collectives (extension, not in MVAPICH2 2.3.7): the blocking calls'
 * algorithms launched on a HIP stream (`stream` is a hipStream_t) behind every collective
 * issued before, returning without waiting (mv2h.h *_enqueue).  Device buffers, predefined
 * ops and contiguous predefined types only; MPIX_Enqueue_check reports a peer timeout of a
 * stream-ordered call after its stream has been synchronised.  MPICH 4's MPIX_*_enqueue
 * take the stream from a stream communicator; here it is an argument of COMM_WORLD calls. */
int MPIX_Allreduce_enqueue(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                           MPI_Op op, MPI_Comm comm, void *stream);
int MPIX_Reduce_enqueue(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                        MPI_Op op, int root, MPI_Comm comm, void *stream);
int MPIX_Reduce_scatter_enqueue(const void *sendbuf, void *recvbuf, const int recvcounts[],
                                MPI_Datatype datatype, MPI_Op op, MPI_Comm comm, void *stream);
int MPIX_Allgather_enqueue(const void *sendbuf, int sendcount, MPI_Datatype sendtype,
                           void *recvbuf, int recvcount, MPI_Datatype recvtype, MPI_Comm comm,
                           void *stream);
int MPIX_Bcast_enqueue(void *buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm,
                       void *stream);
int MPIX_Enqueue_check(MPI_Comm comm);

/* ---- point-to-point on device or host buffers, COMM_WORLD of one node (MPI-3.1 3.2-3.7) ---- */
int MPI_Send(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Recv(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
             MPI_Status *status);
int MPI_Sendrecv(const void *sendbuf, int sendcount, MPI_Datatype sendtype, int dest, int sendtag,
                 void *recvbuf, int recvcount, MPI_Datatype recvtype, int source, int recvtag,
                 MPI_Comm comm, MPI_Status *status);
int MPI_Isend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
              MPI_Request *request);
int MPI_Irecv(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
              MPI_Request *request);
int MPI_Get_count(const MPI_Status *status, MPI_Datatype datatype, int *count);

/* ---- user operations ---- */
int MPI_Op_create(MPI_User_function *user_fn, int commute, MPI_Op *op);
int MPI_Op_free(MPI_Op *op);
int MPI_Op_commutative(MPI_Op op, int *commute);

/* ---- datatypes ---- */
int MPI_Type_size(MPI_Datatype datatype, int *size);
int MPI_Type_get_extent(MPI_Datatype datatype, MPI_Aint *lb, MPI_Aint *extent);
int MPI_Type_get_true_extent(MPI_Datatype datatype, MPI_Aint *true_lb, MPI_Aint *true_extent);
int MPI_Type_contiguous(int count, MPI_Datatype oldtype, MPI_Datatype *newtype);
int MPI_Type_vector(int count, int blocklength, int stride, MPI_Datatype oldtype,
                    MPI_Datatype *newtype);
int MPI_Type_create_hvector(int count, int blocklength, MPI_Aint stride, MPI_Datatype oldtype,
                            MPI_Datatype *newtype);
int MPI_Type_create_indexed_block(int count, int blocklength, const int displacements[],
                                  MPI_Datatype oldtype, MPI_Datatype *newtype);
int MPI_Type_create_hindexed_block(int count, int blocklength, const MPI_Aint displacements[],
                                   MPI_Datatype oldtype, MPI_Datatype *newtype);
int MPI_Type_indexed(int count, const int blocklengths[], const int displacements[],
                     MPI_Datatype oldtype, MPI_Datatype *newtype);
int MPI_Type_create_hindexed(int count, const int blocklengths[], const MPI_Aint displacements[],
                             MPI_Datatype oldtype, MPI_Datatype *newtype);
int MPI_Type_create_struct(int count, const int blocklengths[], const MPI_Aint displacements[],
                           const MPI_Datatype types[], MPI_Datatype *newtype);
int MPI_Type_create_resized(MPI_Datatype oldtype, MPI_Aint lb, MPI_Aint extent, MPI_Datatype *newtype);
int MPI_Type_dup(MPI_Datatype oldtype, MPI_Datatype *newtype);
int MPI_Type_create_subarray(int ndims, const int sizes[], const int subsizes[], const int starts[],
                             int order, MPI_Datatype oldtype, MPI_Datatype *newtype);
int MPI_Type_commit(MPI_Datatype *datatype);
int MPI_Type_free(MPI_Datatype *datatype);
int MPI_Pack(const void *inbuf, int incount, MPI_Datatype datatype, void *outbuf, int outsize,
             int *position, MPI_Comm comm);
int MPI_Unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount,
               MPI_Datatype datatype, MPI_Comm comm);
int MPI_Pack_size(int incount, MPI_Datatype datatype, MPI_Comm comm, int *size);

/* ---- profiling interface (weak MPI_ aliases point here) ---- */
int PMPI_Init(int *argc, char ***argv);
int PMPI_Init_thread(int *argc, char ***argv, int required, int *provided);
int PMPI_Finalize(void);
int PMPI_Initialized(int *flag);
int PMPI_Finalized(int *flag);
int PMPI_Abort(MPI_Comm comm, int errorcode);
double PMPI_Wtime(void);
double PMPI_Wtick(void);
int PMPI_Get_processor_name(char *name, int *resultlen);
int PMPI_Error_string(int errorcode, char *string, int *resultlen);
int PMPI_Error_class(int errorcode, int *errorclass);
int PMPI_Comm_set_errhandler(MPI_Comm comm, MPI_Errhandler errhandler);
int PMPI_Comm_get_errhandler(MPI_Comm comm, MPI_Errhandler *errhandler);
int PMPI_Errhandler_set(MPI_Comm comm, MPI_Errhandler errhandler);
int PMPI_Comm_rank(MPI_Comm comm, int *rank);
int PMPI_Comm_size(MPI_Comm comm, int *size);
int PMPI_Barrier(MPI_Comm comm);
int PMPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype,
                      MPI_Op op);
int PMPI_Allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                   MPI_Op op, MPI_Comm comm);
int PMPI_Reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                int root, MPI_Comm comm);
int PMPI_Reduce_scatter(const void *sendbuf, void *recvbuf, const int recvcounts[],
                        MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
int PMPI_Reduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount,
                              MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);
int PMPI_Allgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf,
                   int recvcount, MPI_Datatype recvtype, MPI_Comm comm);
int PMPI_Bcast(void *buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm);
int PMPI_Iallreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                   MPI_Op op, MPI_Comm comm, MPI_Request *request);
int PMPI_Ireduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                int root, MPI_Comm comm, MPI_Request *request);
int PMPI_Ireduce_scatter(const void *sendbuf, void *recvbuf, const int recvcounts[],
                        MPI_Datatype datatype, MPI_Op op, MPI_Comm comm, MPI_Request *request);
int PMPI_Ireduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount,
                              MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                              MPI_Request *request);
int PMPI_Iallgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf,
                   int recvcount, MPI_Datatype recvtype, MPI_Comm comm, MPI_Request *request);
int PMPIX_Allreduce_enqueue(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                            MPI_Op op, MPI_Comm comm, void *stream);
int PMPIX_Reduce_enqueue(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                         MPI_Op op, int root, MPI_Comm comm, void *stream);
int PMPIX_Reduce_scatter_enqueue(const void *sendbuf, void *recvbuf, const int recvcounts[],
                                 MPI_Datatype datatype, MPI_Op op, MPI_Comm comm, void *stream);
int PMPIX_Allgather_enqueue(const void *sendbuf, int sendcount, MPI_Datatype sendtype,
                            void *recvbuf, int recvcount, MPI_Datatype recvtype, MPI_Comm comm,
                            void *stream);
int PMPIX_Bcast_enqueue(void *buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm,
                        void *stream);
int PMPIX_Enqueue_check(MPI_Comm comm);
int PMPI_Ibcast(void *buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm,
               MPI_Request *request);
int PMPI_Ibarrier(MPI_Comm comm, MPI_Request *request);
int PMPI_Wait(MPI_Request *request, MPI_Status *status);
int PMPI_Test(MPI_Request *request, int *flag, MPI_Status *status);
int PMPI_Waitall(int count, MPI_Request requests[], MPI_Status statuses[]);
int PMPI_Testall(int count, MPI_Request requests[], int *flag, MPI_Status statuses[]);
int PMPI_Request_free(MPI_Request *request);

int PMPI_Send(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int PMPI_Recv(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
             MPI_Status *status);
int PMPI_Sendrecv(const void *sendbuf, int sendcount, MPI_Datatype sendtype, int dest, int sendtag,
                 void *recvbuf, int recvcount, MPI_Datatype recvtype, int source, int recvtag,
                 MPI_Comm comm, MPI_Status *status);
int PMPI_Isend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
              MPI_Request *request);
int PMPI_Irecv(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
              MPI_Request *request);
int PMPI_Get_count(const MPI_Status *status, MPI_Datatype datatype, int *count);
int PMPI_Op_create(MPI_User_function *user_fn, int commute, MPI_Op *op);
int PMPI_Op_free(MPI_Op *op);
int PMPI_Op_commutative(MPI_Op op, int *commute);
int PMPI_Type_size(MPI_Datatype datatype, int *size);
int PMPI_Type_get_extent(MPI_Datatype datatype, MPI_Aint *lb, MPI_Aint *extent);
int PMPI_Type_get_true_extent(MPI_Datatype datatype, MPI_Aint *true_lb, MPI_Aint *true_extent);
int PMPI_Type_contiguous(int count, MPI_Datatype oldtype, MPI_Datatype *newtype);
int PMPI_Type_vector(int count, int blocklength, int stride, MPI_Datatype oldtype,
                     MPI_Datatype *newtype);
int PMPI_Type_create_hvector(int count, int blocklength, MPI_Aint stride, MPI_Datatype oldtype,
                             MPI_Datatype *newtype);
int PMPI_Type_create_indexed_block(int count, int blocklength, const int displacements[],
                                   MPI_Datatype oldtype, MPI_Datatype *newtype);
int PMPI_Type_create_hindexed_block(int count, int blocklength, const MPI_Aint displacements[],
                                   MPI_Datatype oldtype, MPI_Datatype *newtype);
int PMPI_Type_indexed(int count, const int blocklengths[], const int displacements[],
                     MPI_Datatype oldtype, MPI_Datatype *newtype);
int PMPI_Type_create_hindexed(int count, const int blocklengths[], const MPI_Aint displacements[],
                             MPI_Datatype oldtype, MPI_Datatype *newtype);
int PMPI_Type_create_struct(int count, const int blocklengths[], const MPI_Aint displacements[],
                           const MPI_Datatype types[], MPI_Datatype *newtype);
int PMPI_Type_create_resized(MPI_Datatype oldtype, MPI_Aint lb, MPI_Aint extent, MPI_Datatype *newtype);
int PMPI_Type_dup(MPI_Datatype oldtype, MPI_Datatype *newtype);
int PMPI_Type_create_subarray(int ndims, const int sizes[], const int subsizes[], const int starts[],
                             int order, MPI_Datatype oldtype, MPI_Datatype *newtype);
int PMPI_Type_commit(MPI_Datatype *datatype);
int PMPI_Type_free(MPI_Datatype *datatype);
int PMPI_Pack(const void *inbuf, int incount, MPI_Datatype datatype, void *outbuf, int outsize,
              int *position, MPI_Comm comm);
int PMPI_Unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount,
                MPI_Datatype datatype, MPI_Comm comm);
int PMPI_Pack_size(int incount, MPI_Datatype datatype, MPI_Comm comm, int *size);
int PMPI_T_init_thread(int required, int *provided);
int PMPI_T_finalize(void);
int PMPI_T_enum_get_info(MPI_T_enum enumtype, int *num, char *name, int *name_len);
int PMPI_T_enum_get_item(MPI_T_enum enumtype, int indx, int *value, char *name, int *name_len);
int PMPI_T_cvar_get_num(int *num_cvar);
int PMPI_T_cvar_get_info(int cvar_index, char *name, int *name_len, int *verbosity, MPI_Datatype *datatype,
                        MPI_T_enum *enumtype, char *desc, int *desc_len, int *binding, int *scope);
int PMPI_T_cvar_get_index(const char *name, int *cvar_index);
int PMPI_T_cvar_handle_alloc(int cvar_index, void *obj_handle, MPI_T_cvar_handle *handle, int *count);
int PMPI_T_cvar_handle_free(MPI_T_cvar_handle *handle);
int PMPI_T_cvar_read(MPI_T_cvar_handle handle, void *buf);
int PMPI_T_cvar_write(MPI_T_cvar_handle handle, const void *buf);
int PMPI_T_pvar_get_num(int *num_pvar);
int PMPI_T_pvar_get_info(int pvar_index, char *name, int *name_len, int *verbosity, int *var_class,
                        MPI_Datatype *datatype, MPI_T_enum *enumtype, char *desc, int *desc_len, int *binding,
                        int *readonly, int *continuous, int *atomic);
int PMPI_T_pvar_get_index(const char *name, int var_class, int *pvar_index);
int PMPI_T_pvar_session_create(MPI_T_pvar_session *session);
int PMPI_T_pvar_session_free(MPI_T_pvar_session *session);
int PMPI_T_pvar_handle_alloc(MPI_T_pvar_session session, int pvar_index, void *obj_handle, MPI_T_pvar_handle *handle,
                            int *count);
int PMPI_T_pvar_handle_free(MPI_T_pvar_session session, MPI_T_pvar_handle *handle);
int PMPI_T_pvar_start(MPI_T_pvar_session session, MPI_T_pvar_handle handle);
int PMPI_T_pvar_stop(MPI_T_pvar_session session, MPI_T_pvar_handle handle);
int PMPI_T_pvar_read(MPI_T_pvar_session session, MPI_T_pvar_handle handle, void *buf);
int PMPI_T_pvar_write(MPI_T_pvar_session session, MPI_T_pvar_handle handle, const void *buf);
int PMPI_T_pvar_reset(MPI_T_pvar_session session, MPI_T_pvar_handle handle);
int PMPI_T_pvar_readreset(MPI_T_pvar_session session, MPI_T_pvar_handle handle, void *buf);
int PMPI_T_category_get_num(int *num_cat);
int PMPI_T_category_get_info(int cat_index, char *name, int *name_len, char *desc, int *desc_len, int *num_cvars,
                            int *num_pvars, int *num_categories);
int PMPI_T_category_get_index(const char *name, int *cat_index);
int PMPI_T_category_get_cvars(int cat_index, int len, int indices[]);
int PMPI_T_category_get_pvars(int cat_index, int len, int indices[]);
int PMPI_T_category_get_categories(int cat_index, int len, int indices[]);
int PMPI_T_category_changed(int *stamp);

#ifdef __cplusplus
}
#endif

#endif /* MV2AMD_MPI_H_INCLUDED */
