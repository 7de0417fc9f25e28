// mpi_api.cpp — the MPI-3.1 C entry points (include/mpi.h) over the mv2h
// C-ABI.  Argument checking and error-handler behaviour follow the
// reference's MPI layer (e.g. allreduce.c:827-960, reduce_local.c:206-268):
// count == 0 returns immediately, a predefined op on a type outside its
// groups is MPI_ERR_OP, errors go through the communicator's error handler
// (default MPI_ERRORS_ARE_FATAL).  Every MPI_X is a weak alias of PMPI_X
// (allreduce.c:80-84).
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../../include/mpi.h"
#include "../../../include/mv2h.h"
#include "../../../include/mpir_op.h"
#include "../common.h"
#include "../runtime/log.h"
#include "../runtime/orders.h"
#include "../runtime/pvars.h"
#include "../runtime/world.h"
#include "datatype.h"
#include "user_coll.h"

using namespace mv2;

extern "C" int PMPI_Type_get_extent(MPI_Datatype dt, MPI_Aint *lb, MPI_Aint *extent);

namespace {

std::recursive_mutex g_cs;  // global critical section (allreduce.c:838)
MPI_Errhandler g_eh[2] = {MPI_ERRORS_ARE_FATAL, MPI_ERRHANDLER_NULL};  // SELF: unset, WORLD's applies
bool g_initialized = false, g_finalized = false;

struct UserOp {
    MPI_User_function *fn;
    int commute;
    bool live;
};
std::vector<UserOp> g_uops;
constexpr int kUserOpBase = (int)0x98000000;  // direct-kind op handles (MPICH kind bits 10, object 0x18)

const char *err_name(int c) {
    switch (c) {
    case MPI_SUCCESS: return "MPI_SUCCESS: no error";
    case MPI_ERR_BUFFER: return "MPI_ERR_BUFFER: invalid buffer pointer";
    case MPI_ERR_COUNT: return "MPI_ERR_COUNT: invalid count argument";
    case MPI_ERR_TYPE: return "MPI_ERR_TYPE: invalid datatype";
    case MPI_ERR_COMM: return "MPI_ERR_COMM: invalid communicator";
    case MPI_ERR_ROOT: return "MPI_ERR_ROOT: invalid root";
    case MPI_ERR_OP: return "MPI_ERR_OP: invalid reduce operation";
    case MPI_ERR_ARG: return "MPI_ERR_ARG: invalid argument";
    case MPI_ERR_TRUNCATE: return "MPI_ERR_TRUNCATE: message truncated";
    case MPI_ERR_OTHER: return "MPI_ERR_OTHER: other error";
    case MPI_ERR_INTERN: return "MPI_ERR_INTERN: internal error";
    case MPI_ERR_NO_MEM: return "MPI_ERR_NO_MEM: out of memory";
    case MPI_ERR_UNSUPPORTED_OPERATION: return "MPI_ERR_UNSUPPORTED_OPERATION: unsupported operation";
    default: return "unknown error";
    }
}

int comm_index(MPI_Comm c) {
    if (c == MPI_COMM_WORLD) return 0;
    if (c == MPI_COMM_SELF) return 1;
    return -1;
}

// MPIR_Err_return_comm (allreduce.c:956, errutil.c:249-289): fatal handler aborts, return
// handler passes the code; an invalid communicator, or one whose handler was never set
// (MPI_COMM_SELF's until MPI_Comm_set_errhandler), takes MPI_COMM_WORLD's handler
int err_return(MPI_Comm comm, int code, const char *fn) {
    if (code == MPI_SUCCESS) return code;
    const int ci = comm_index(comm);
    const MPI_Errhandler eh = ci >= 0 && g_eh[ci] != MPI_ERRHANDLER_NULL ? g_eh[ci] : g_eh[0];
    if (eh == MPI_ERRORS_ARE_FATAL) {
        fprintf(stderr, "[mv2amd rank %d] Fatal error in %s: %s\n", mv2h_rank(), fn, err_name(code));
        fflush(stderr);
        abort();
    }
    static const int verbose = [] {
        const char *v = getenv("MV2AMD_ERR_VERBOSE");  // tests: name every error a call returns
        return v && *v && *v != '0';
    }();
    if (verbose) {
        fprintf(stderr, "[mv2amd rank %d] %s returned %s\n", mv2h_rank(), fn, err_name(code));
        fflush(stderr);
    }
    return code;
}

UserOp *user_op(MPI_Op op) {
    const unsigned idx = (unsigned)(op - kUserOpBase);
    if ((op & 0xff000000) != (kUserOpBase & 0xff000000) || idx >= g_uops.size() || !g_uops[idx].live) return nullptr;
    return &g_uops[idx];
}

bool op_valid(MPI_Op op) { return is_builtin_op(op) || user_op(op) != nullptr; }

bool is_dev(const void *p) { return p && p != MPI_IN_PLACE && mv2h_is_device_ptr(p); }

// ---- user-op path: user functions are host callbacks (the reference also
// calls them on host copies of device buffers, reduce_local.c:54-164); the
// collectives' host evaluation is user_coll.cpp ----
int copy_to_host(HostBuf &h, const void *p, size_t bytes) {
    h.resize(bytes ? bytes : 1);
    if (!h.data()) return MPI_ERR_NO_MEM;
    if (is_dev(p)) return mv2h_memcpy_dtoh(h.data(), p, bytes);
    memcpy(h.data(), p, bytes);
    return 0;
}
int copy_from_host(void *p, const HostBuf &h, size_t bytes) {
    if (is_dev(p)) return mv2h_memcpy_htod(p, h.data(), bytes);
    memcpy(p, h.data(), bytes);
    return 0;
}

// ---- x87 80-bit long double (MPI_LONG_DOUBLE, MPI_C_LONG_DOUBLE_COMPLEX,
// MPI_LONG_DOUBLE_INT): gfx950 has no 80-bit float, so these builtin ops run
// on the host, as the reference's own loops do (oputil.h:316-349,
// opmaxloc.c:65-87), through the same algorithm plans as user ops.  Only
// these three types take this path; every other builtin type is reduced on
// the GPU and has no host path.
int g_ld_op = -1;  // op index of the current x87 call (set under the global critical section)

template <class T>
inline T x_max(T a, T b) { return (a != a && b != b) ? a : (a != a) ? b : (b != b) ? a : ((b > a) ? b : a); }
template <class T>
inline T x_min(T a, T b) { return (a != a && b != b) ? a : (a != a) ? b : (b != b) ? a : ((a > b) ? b : a); }

struct LdInt {
    long double value;
    int loc;
};

void ld_uop(void *in, void *inout, int *len, MPI_Datatype *dt) {
    const long n = *len;
    const int op = g_ld_op;
    if (*dt == MPI_LONG_DOUBLE) {
        const long double *b = (const long double *)in;
        long double *a = (long double *)inout;
        for (long i = 0; i < n; ++i) {
            switch (op) {
            case OP_SUM: a[i] = a[i] + b[i]; break;
            case OP_PROD: a[i] = a[i] * b[i]; break;
            case OP_MAX: a[i] = x_max(a[i], b[i]); break;
            case OP_MIN: a[i] = x_min(a[i], b[i]); break;
            case OP_LAND: a[i] = (a[i] && b[i]); break;
            case OP_LOR: a[i] = (a[i] || b[i]); break;
            case OP_LXOR: a[i] = ((a[i] && !b[i]) || (!a[i] && b[i])); break;
            case OP_REPLACE: a[i] = b[i]; break;
            default: break;
            }
        }
    } else if (*dt == MPI_C_LONG_DOUBLE_COMPLEX) {
        const __complex__ long double *b = (const __complex__ long double *)in;
        __complex__ long double *a = (__complex__ long double *)inout;
        for (long i = 0; i < n; ++i) {
            if (op == OP_SUM) a[i] = a[i] + b[i];
            else if (op == OP_PROD) a[i] = a[i] * b[i];  // Annex G __mulxc3, like the reference's C99 loop
            else if (op == OP_REPLACE) a[i] = b[i];
        }
    } else if (*dt == MPI_LONG_DOUBLE_INT) {
        const LdInt *b = (const LdInt *)in;
        LdInt *a = (LdInt *)inout;
        for (long i = 0; i < n; ++i) {
            if (op == OP_REPLACE) {
                memcpy(&a[i].value, &b[i].value, 10);
                a[i].loc = b[i].loc;
                continue;
            }
            if (op != OP_MAXLOC && op != OP_MINLOC) continue;
            const long double av = a[i].value, bv = b[i].value;
            if (av != av && bv != bv) {
                a[i].loc = std::min(a[i].loc, b[i].loc);
            } else if (av != av) {
                a[i].value = bv;
                a[i].loc = b[i].loc;
            } else if (bv != bv) {
            } else if (op == OP_MAXLOC ? av < bv : av > bv) {
                a[i].value = bv;
                a[i].loc = b[i].loc;
            } else if (op == OP_MAXLOC ? av <= bv : av >= bv) {
                a[i].loc = std::min(a[i].loc, b[i].loc);
            }
        }
    }
}

bool is_x87(MPI_Datatype dt) {
    return dt == MPI_LONG_DOUBLE || dt == MPI_C_LONG_DOUBLE_COMPLEX || dt == MPI_LONG_DOUBLE_INT;
}

int user_reduce_local(const void *in, void *inout, int count, MPI_Datatype dt, UserOp *u) {
    long span = dtype_span(dt, count);
    if (span < 0) return MPI_ERR_TYPE;
    HostBuf hin(HS_IN), hio(HS_INOUT);
    int rc = copy_to_host(hin, in, span);
    if (!rc) rc = copy_to_host(hio, inout, span);
    if (rc) return MPI_ERR_OTHER;
    int c = count;
    MPI_Datatype d = dt;
    u->fn(hin.data(), hio.data(), &c, &d);
    return copy_from_host(inout, hio, span) ? MPI_ERR_OTHER : MPI_SUCCESS;
}

// one MPI_T-counted call (runtime/pvars.h)
int user_allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, UserOp *u, int opk) {
    pvar_begin();
    const int rc = host_allreduce(sendbuf, recvbuf, count, dt, HostOp{u->fn, opk});
    pvar_end(rc == MPI_SUCCESS);
    return rc;
}

// one MPI_T-counted call (runtime/pvars.h)
int user_reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, UserOp *u, int root, int opk) {
    pvar_begin();
    const int rc = host_reduce(sendbuf, recvbuf, count, dt, HostOp{u->fn, opk}, root);
    pvar_end(rc == MPI_SUCCESS);
    return rc;
}

}  // namespace

extern "C" int PMPI_Type_get_extent(MPI_Datatype dt, MPI_Aint *lb, MPI_Aint *extent);

namespace {

// one MPI_T-counted call (runtime/pvars.h)
int user_reduce_scatter(const void *sendbuf, void *recvbuf, const int *counts, MPI_Datatype dt, UserOp *u, int opk) {
    pvar_begin();
    const int rc = host_reduce_scatter(sendbuf, recvbuf, counts, dt, HostOp{u->fn, opk});
    pvar_end(rc == MPI_SUCCESS);
    return rc;
}

}  // namespace

#define WEAK(name) __attribute__((weak, alias("P" #name)))

extern "C" {

// ---------------------------------------------------------------- environment
int PMPI_Init(int *, char ***) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    if (g_initialized) return err_return(MPI_COMM_WORLD, MPI_ERR_OTHER, "MPI_Init");
    int rc = world_init();
    if (rc) return err_return(MPI_COMM_WORLD, rc, "MPI_Init");
    g_initialized = true;
    return MPI_SUCCESS;
}
int MPI_Init(int *argc, char ***argv) WEAK(MPI_Init);

int PMPI_Init_thread(int *argc, char ***argv, int required, int *provided) {
    int rc = PMPI_Init(argc, argv);
    if (provided) *provided = required > MPI_THREAD_SERIALIZED ? MPI_THREAD_SERIALIZED : required;
    return rc;
}
int MPI_Init_thread(int *argc, char ***argv, int required, int *provided) WEAK(MPI_Init_thread);

int PMPI_Finalize(void) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    world_finalize();
    g_finalized = true;
    return MPI_SUCCESS;
}
int MPI_Finalize(void) WEAK(MPI_Finalize);

int PMPI_Initialized(int *flag) {
    *flag = g_initialized ? 1 : 0;
    return MPI_SUCCESS;
}
int MPI_Initialized(int *flag) WEAK(MPI_Initialized);

int PMPI_Finalized(int *flag) {
    *flag = g_finalized ? 1 : 0;
    return MPI_SUCCESS;
}
int MPI_Finalized(int *flag) WEAK(MPI_Finalized);

int PMPI_Abort(MPI_Comm, int errorcode) {
    fprintf(stderr, "[mv2amd rank %d] MPI_Abort(%d)\n", mv2h_rank(), errorcode);
    fflush(stderr);
    _exit(errorcode ? errorcode : 1);
}
int MPI_Abort(MPI_Comm comm, int errorcode) WEAK(MPI_Abort);

double PMPI_Wtime(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * ts.tv_nsec;
}
double MPI_Wtime(void) WEAK(MPI_Wtime);

double PMPI_Wtick(void) { return 1e-9; }
double MPI_Wtick(void) WEAK(MPI_Wtick);

int PMPI_Get_processor_name(char *name, int *len) {
    gethostname(name, MPI_MAX_PROCESSOR_NAME);
    name[MPI_MAX_PROCESSOR_NAME - 1] = 0;
    *len = (int)strlen(name);
    return MPI_SUCCESS;
}
int MPI_Get_processor_name(char *name, int *len) WEAK(MPI_Get_processor_name);

int PMPI_Error_string(int code, char *s, int *len) {
    snprintf(s, MPI_MAX_ERROR_STRING, "%s", err_name(code));
    *len = (int)strlen(s);
    return MPI_SUCCESS;
}
int MPI_Error_string(int code, char *s, int *len) WEAK(MPI_Error_string);

int PMPI_Error_class(int code, int *cls) {
    *cls = code & 0x7f;
    return MPI_SUCCESS;
}
int MPI_Error_class(int code, int *cls) WEAK(MPI_Error_class);

int PMPI_Comm_set_errhandler(MPI_Comm comm, MPI_Errhandler eh) {
    const int ci = comm_index(comm);
    if (ci < 0) return MPI_ERR_COMM;
    if (eh != MPI_ERRORS_ARE_FATAL && eh != MPI_ERRORS_RETURN) return MPI_ERR_ARG;
    g_eh[ci] = eh;
    return MPI_SUCCESS;
}
int MPI_Comm_set_errhandler(MPI_Comm comm, MPI_Errhandler eh) WEAK(MPI_Comm_set_errhandler);

int PMPI_Errhandler_set(MPI_Comm comm, MPI_Errhandler eh) { return PMPI_Comm_set_errhandler(comm, eh); }
int MPI_Errhandler_set(MPI_Comm comm, MPI_Errhandler eh) WEAK(MPI_Errhandler_set);

int PMPI_Comm_get_errhandler(MPI_Comm comm, MPI_Errhandler *eh) {
    const int ci = comm_index(comm);
    if (ci < 0) return MPI_ERR_COMM;
    *eh = g_eh[ci] == MPI_ERRHANDLER_NULL ? MPI_ERRORS_ARE_FATAL : g_eh[ci];  // comm_get_errhandler.c: unset reads FATAL
    return MPI_SUCCESS;
}
int MPI_Comm_get_errhandler(MPI_Comm comm, MPI_Errhandler *eh) WEAK(MPI_Comm_get_errhandler);

// ---------------------------------------------------------------- communicators
int PMPI_Comm_rank(MPI_Comm comm, int *rank) {
    const int ci = comm_index(comm);
    if (ci < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_COMM, "MPI_Comm_rank");
    *rank = ci == 0 ? mv2h_rank() : 0;
    return MPI_SUCCESS;
}
int MPI_Comm_rank(MPI_Comm comm, int *rank) WEAK(MPI_Comm_rank);

int PMPI_Comm_size(MPI_Comm comm, int *size) {
    const int ci = comm_index(comm);
    if (ci < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_COMM, "MPI_Comm_size");
    *size = ci == 0 ? mv2h_size() : 1;
    return MPI_SUCCESS;
}
int MPI_Comm_size(MPI_Comm comm, int *size) WEAK(MPI_Comm_size);

int PMPI_Barrier(MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const int ci = comm_index(comm);
    if (ci < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_COMM, "MPI_Barrier");
    if (ci == 0 && mv2h_barrier()) return err_return(comm, MPI_ERR_OTHER, "MPI_Barrier");
    return MPI_SUCCESS;
}
int MPI_Barrier(MPI_Comm comm) WEAK(MPI_Barrier);

// ---------------------------------------------------------------- user ops
int PMPI_Op_create(MPI_User_function *fn, int commute, MPI_Op *op) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    if (!fn || !op) return err_return(MPI_COMM_WORLD, MPI_ERR_ARG, "MPI_Op_create");
    g_uops.push_back(UserOp{fn, commute ? 1 : 0, true});
    *op = kUserOpBase + (int)(g_uops.size() - 1);
    return MPI_SUCCESS;
}
int MPI_Op_create(MPI_User_function *fn, int commute, MPI_Op *op) WEAK(MPI_Op_create);

int PMPI_Op_free(MPI_Op *op) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    UserOp *u = op ? user_op(*op) : nullptr;
    if (!u) return err_return(MPI_COMM_WORLD, MPI_ERR_OP, "MPI_Op_free");
    u->live = false;
    *op = MPI_OP_NULL;
    return MPI_SUCCESS;
}
int MPI_Op_free(MPI_Op *op) WEAK(MPI_Op_free);

int PMPI_Op_commutative(MPI_Op op, int *commute) {
    if (is_builtin_op(op)) {
        *commute = 1;
        return MPI_SUCCESS;
    }
    UserOp *u = user_op(op);
    if (!u) return err_return(MPI_COMM_WORLD, MPI_ERR_OP, "MPI_Op_commutative");
    *commute = u->commute;
    return MPI_SUCCESS;
}
int MPI_Op_commutative(MPI_Op op, int *commute) WEAK(MPI_Op_commutative);

// ---------------------------------------------------------------- reductions
// A builtin op on `count` elements of a builtin type (device or host buffers;
// x87 types on the host): the MPI error class, no error handler.
static int builtin_reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype dt, MPI_Op op) {
    if (!dtype_is_builtin(dt)) return MPI_ERR_OP;
    if (is_x87(dt)) {
        if (mv2h_op_check(op, dt)) return MPI_ERR_OP;
        UserOp x{ld_uop, 1, true};
        g_ld_op = op_index(op);
        return op_index(op) == OP_NO_OP ? 0 : user_reduce_local(inbuf, inoutbuf, count, dt, &x);
    }
    return mv2h_reduce_local(inbuf, inoutbuf, (size_t)count, dt, op, nullptr);
}

int PMPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype dt, MPI_Op op) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPI_Reduce_local";
    if (count < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_COUNT, fn);
    if (!op_valid(op)) return err_return(MPI_COMM_WORLD, MPI_ERR_OP, fn);
    if (!dtype_valid(dt)) return err_return(MPI_COMM_WORLD, MPI_ERR_TYPE, fn);
    if (!dtype_committed(dt)) return err_return(MPI_COMM_WORLD, MPI_ERR_TYPE, fn);
    if (count == 0) return MPI_SUCCESS;
    // reduce_local.c:233-237: aliased operands (MPIR_ERRTEST_ALIAS_COLL), then MPI_IN_PLACE
    if (inbuf == inoutbuf || inbuf == MPI_IN_PLACE || inoutbuf == MPI_IN_PLACE)
        return err_return(MPI_COMM_WORLD, MPI_ERR_BUFFER, fn);
    if (UserOp *u = user_op(op)) return err_return(MPI_COMM_WORLD, user_reduce_local(inbuf, inoutbuf, count, dt, u), fn);
    return err_return(MPI_COMM_WORLD, builtin_reduce_local(inbuf, inoutbuf, count, dt, op), fn);
}
int MPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype dt, MPI_Op op) WEAK(MPI_Reduce_local);

// ---------------------------------------------------------------------------
// The predefined ops as MPI_User_function entry points (include/mpir_op.h):
// MPIR_Op_table (allreduce.c:95-100) indexed by MPIR_OP_HDL_TO_FN
// (mpiimpl.h:4031), and the per-op type checks (MPIR_Op_check_dtype_table).
// Unlike the reference's host loops (opsum.c:26-90 ...) they take device
// buffers: one HBM-streaming kernel, synchronous like any MPI_User_function;
// host buffers are staged as for MPI_Reduce_local.  A type the op does not
// accept leaves inoutvec untouched and sets the error MPIR_Op_errno returns
// (the reference keeps it in the thread-private op_errno, opsum.c:82-86).
// ---------------------------------------------------------------------------
static thread_local int t_op_errno = MPI_SUCCESS;

static void op_entry(MPI_Op op, void *invec, void *inoutvec, int *len, MPI_Datatype *type) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    if (!len || !type || *len < 0) {
        t_op_errno = MPI_ERR_ARG;
        return;
    }
    if (*len == 0) return;
    if (!dtype_valid(*type)) {
        t_op_errno = MPI_ERR_TYPE;
        return;
    }
    if (mv2h_op_check(op, *type)) {
        t_op_errno = MPI_ERR_OP;
        return;
    }
    const int rc = builtin_reduce_local(invec, inoutvec, *len, *type, op);
    if (rc) t_op_errno = rc;
}

#define MV2_OP_FN(NAME, HANDLE)                                                               \
    void NAME(void *invec, void *inoutvec, int *len, MPI_Datatype *type) {                     \
        op_entry(HANDLE, invec, inoutvec, len, type);                                          \
    }                                                                                          \
    int NAME##_check_dtype(MPI_Datatype type) {                                                \
        return !dtype_valid(type) ? MPI_ERR_TYPE : (mv2h_op_check(HANDLE, type) ? MPI_ERR_OP : MPI_SUCCESS); \
    }
MV2_OP_FN(MPIR_MAXF, MPI_MAX)
MV2_OP_FN(MPIR_MINF, MPI_MIN)
MV2_OP_FN(MPIR_SUM, MPI_SUM)
MV2_OP_FN(MPIR_PROD, MPI_PROD)
MV2_OP_FN(MPIR_LAND, MPI_LAND)
MV2_OP_FN(MPIR_BAND, MPI_BAND)
MV2_OP_FN(MPIR_LOR, MPI_LOR)
MV2_OP_FN(MPIR_BOR, MPI_BOR)
MV2_OP_FN(MPIR_LXOR, MPI_LXOR)
MV2_OP_FN(MPIR_BXOR, MPI_BXOR)
MV2_OP_FN(MPIR_MINLOC, MPI_MINLOC)
MV2_OP_FN(MPIR_MAXLOC, MPI_MAXLOC)
MV2_OP_FN(MPIR_REPLACE, MPI_REPLACE)
MV2_OP_FN(MPIR_NO_OP, MPI_NO_OP)
#undef MV2_OP_FN

// order of the predefined op handles' low nibble (mpi.h: MPI_MAX = ...01 .. MPI_NO_OP = ...0e)
MPI_User_function *MPIR_Op_table[] = {MPIR_MAXF, MPIR_MINF, MPIR_SUM,  MPIR_PROD,   MPIR_LAND,   MPIR_BAND,    MPIR_LOR,
                                      MPIR_BOR,  MPIR_LXOR, MPIR_BXOR, MPIR_MINLOC, MPIR_MAXLOC, MPIR_REPLACE, MPIR_NO_OP};
MPIR_Op_check_dtype_fn *MPIR_Op_check_dtype_table[] = {
    MPIR_MAXF_check_dtype, MPIR_MINF_check_dtype,   MPIR_SUM_check_dtype,    MPIR_PROD_check_dtype,
    MPIR_LAND_check_dtype, MPIR_BAND_check_dtype,   MPIR_LOR_check_dtype,    MPIR_BOR_check_dtype,
    MPIR_LXOR_check_dtype, MPIR_BXOR_check_dtype,   MPIR_MINLOC_check_dtype, MPIR_MAXLOC_check_dtype,
    MPIR_REPLACE_check_dtype, MPIR_NO_OP_check_dtype};

int MPIR_Op_errno(void) {
    const int e = t_op_errno;
    t_op_errno = MPI_SUCCESS;
    return e;
}

// The buffer checks of the reference's MPI layer, MPI_ERR_BUFFER each (mpierrs.h):
// MPIR_ERRTEST_USERBUFFER (:313-331) — no buffer for count > 0 elements of a builtin type, or of
// a derived type whose true lb is 0 and size > 0 (a null buffer is MPI_BOTTOM otherwise);
// MPIR_ERRTEST_{SEND,RECV,}BUF_INPLACE (:274-301) — MPI_IN_PLACE where the call has no in-place
// form; MPIR_ERRTEST_ALIAS_COLL (:132-140, MPIR_CVAR_COLL_ALIAS_CHECK's default 1) — the send
// buffer is the receive buffer.
static bool null_userbuf(const void *buf, long count, MPI_Datatype dt) {
    if (count <= 0 || buf) return false;
    return dtype_is_builtin(dt) || (dtype_valid(dt) && dtype_true_lb(dt) == 0 && dtype_size(dt) > 0);
}
static bool inplace_buf(const void *buf, long count) { return count > 0 && buf == MPI_IN_PLACE; }

// allreduce.c:880-888
static int allreduce_buf_checks(const void *sendbuf, const void *recvbuf, int count, MPI_Datatype dt) {
    if (count != 0 && sendbuf != MPI_IN_PLACE && sendbuf == recvbuf) return MPI_ERR_BUFFER;
    if (sendbuf != MPI_IN_PLACE && null_userbuf(sendbuf, count, dt)) return MPI_ERR_BUFFER;
    if (inplace_buf(recvbuf, count) || null_userbuf(recvbuf, count, dt)) return MPI_ERR_BUFFER;
    return MPI_SUCCESS;
}

// reduce.c:1190-1202: the receive buffer matters at the root only; elsewhere MPI_IN_PLACE is
// not a send buffer
static int reduce_buf_checks(const void *sendbuf, const void *recvbuf, int count, MPI_Datatype dt, bool at_root) {
    if (sendbuf != MPI_IN_PLACE && null_userbuf(sendbuf, count, dt)) return MPI_ERR_BUFFER;
    if (!at_root) return inplace_buf(sendbuf, count) ? MPI_ERR_BUFFER : MPI_SUCCESS;
    if (inplace_buf(recvbuf, count) || null_userbuf(recvbuf, count, dt)) return MPI_ERR_BUFFER;
    if (count != 0 && sendbuf != MPI_IN_PLACE && sendbuf == recvbuf) return MPI_ERR_BUFFER;
    return MPI_SUCCESS;
}

// red_scat.c:1182-1189 (and red_scat_block.c:1147-1154, the same with every count equal)
static int reduce_scatter_buf_checks(const void *sendbuf, const void *recvbuf, long mine, long sum, MPI_Datatype dt) {
    if (inplace_buf(recvbuf, mine)) return MPI_ERR_BUFFER;
    if (sendbuf != MPI_IN_PLACE && sum != 0 && sendbuf == recvbuf) return MPI_ERR_BUFFER;
    if (null_userbuf(recvbuf, mine, dt) || null_userbuf(sendbuf, sum, dt)) return MPI_ERR_BUFFER;
    return MPI_SUCCESS;
}

// allgather.c:952-958, before any other argument check: the send buffer is this rank's block
// of the receive buffer, the block measured in recvtype's size (as the reference measures it)
static bool allgather_alias(const void *sendbuf, int sendcount, MPI_Datatype sendtype, const void *recvbuf,
                            int recvcount, MPI_Datatype recvtype, int rank) {
    return sendbuf != MPI_IN_PLACE && sendtype == recvtype && recvcount != 0 && sendcount != 0 &&
           dtype_valid(recvtype) && sendbuf == (const char *)recvbuf + (long)rank * recvcount * dtype_size(recvtype);
}

// allgather.c:961-987, after the counts and types
static int allgather_buf_checks(const void *sendbuf, int sendcount, MPI_Datatype sendtype, const void *recvbuf,
                                int recvcount, MPI_Datatype recvtype) {
    if (sendbuf != MPI_IN_PLACE && null_userbuf(sendbuf, sendcount, sendtype)) return MPI_ERR_BUFFER;
    if (inplace_buf(recvbuf, recvcount) || null_userbuf(recvbuf, recvcount, recvtype)) return MPI_ERR_BUFFER;
    return MPI_SUCCESS;
}

// The checks every reduction shares, in allreduce.c:863-899's order: communicator, count,
// datatype, op handle, a derived type committed, then the call's buffer checks (buf_rc,
// computed by the caller), then the op against the type (MPIR_OP_HDL_TO_DTYPE_FN)
static int coll_checks(MPI_Comm comm, int count, MPI_Datatype dt, MPI_Op op, int buf_rc = MPI_SUCCESS) {
    if (!g_initialized || g_finalized) return MPI_ERR_OTHER;
    if (comm_index(comm) < 0) return MPI_ERR_COMM;
    if (count < 0) return MPI_ERR_COUNT;
    if (!dtype_valid(dt)) return MPI_ERR_TYPE;
    if (!op_valid(op)) return MPI_ERR_OP;
    if (!dtype_committed(dt)) return MPI_ERR_TYPE;
    if (buf_rc) return buf_rc;
    if (is_builtin_op(op) && !dtype_is_builtin(dt)) return MPI_ERR_OP;  // e.g. opsum.c:119-121
    if (is_builtin_op(op) && mv2h_op_check(op, dt)) return MPI_ERR_OP;
    return MPI_SUCCESS;
}

static int comm_rank_of(MPI_Comm comm) { return comm == MPI_COMM_SELF ? 0 : mv2h_rank(); }

int PMPI_Allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPI_Allreduce";
    int rc = coll_checks(comm, count, dt, op, allreduce_buf_checks(sendbuf, recvbuf, count, dt));
    if (rc) return err_return(comm, rc, fn);
    if (count == 0) return MPI_SUCCESS;
    if (comm == MPI_COMM_SELF) {
        if (sendbuf != MPI_IN_PLACE && sendbuf != recvbuf) {
            const long span = dtype_span(dt, count);
            rc = is_dev(recvbuf) || is_dev(sendbuf) ? mv2h_memcpy_dtod(recvbuf, sendbuf, span) : (memcpy(recvbuf, sendbuf, span), 0);
        }
        return err_return(comm, rc, fn);
    }
    if (UserOp *u = user_op(op))
        return err_return(comm, user_allreduce(sendbuf, recvbuf, count, dt, u, u->commute ? OPK_USER_COMM : OPK_USER_NONCOMM), fn);
    if (is_x87(dt) && op_index(op) < OP_REPLACE) {
        UserOp x{ld_uop, 1, true};
        g_ld_op = op_index(op);
        return err_return(comm, user_allreduce(sendbuf, recvbuf, count, dt, &x, OPK_BUILTIN), fn);
    }
    rc = mv2h_allreduce(sendbuf, recvbuf, (size_t)count, dt, op, nullptr);
    return err_return(comm, rc, fn);
}
int MPI_Allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, MPI_Comm comm) WEAK(MPI_Allreduce);

int PMPI_Reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, int root, MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPI_Reduce";
    if (!g_initialized || g_finalized) return err_return(comm, MPI_ERR_OTHER, fn);
    if (comm_index(comm) < 0) return err_return(comm, MPI_ERR_COMM, fn);
    int size = comm == MPI_COMM_SELF ? 1 : mv2h_size();
    if (root < 0 || root >= size) return err_return(comm, MPI_ERR_ROOT, fn);  // reduce.c:1178, before the count
    int rc = coll_checks(comm, count, dt, op, reduce_buf_checks(sendbuf, recvbuf, count, dt, comm_rank_of(comm) == root));
    if (rc) return err_return(comm, rc, fn);
    if (count == 0) return MPI_SUCCESS;
    if (comm == MPI_COMM_SELF) {
        if (sendbuf != MPI_IN_PLACE && sendbuf != recvbuf) {
            const long span = dtype_span(dt, count);
            rc = is_dev(recvbuf) || is_dev(sendbuf) ? mv2h_memcpy_dtod(recvbuf, sendbuf, span) : (memcpy(recvbuf, sendbuf, span), 0);
        }
        return err_return(comm, rc, fn);
    }
    if (UserOp *u = user_op(op))
        return err_return(comm, user_reduce(sendbuf, recvbuf, count, dt, u, root, u->commute ? OPK_USER_COMM : OPK_USER_NONCOMM), fn);
    if (is_x87(dt) && op_index(op) < OP_REPLACE) {
        UserOp x{ld_uop, 1, true};
        g_ld_op = op_index(op);
        return err_return(comm, user_reduce(sendbuf, recvbuf, count, dt, &x, root, OPK_BUILTIN), fn);
    }
    rc = mv2h_reduce(sendbuf, recvbuf, (size_t)count, dt, op, root, nullptr);
    return err_return(comm, rc, fn);
}
int MPI_Reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, int root, MPI_Comm comm) WEAK(MPI_Reduce);

int PMPI_Reduce_scatter(const void *sendbuf, void *recvbuf, const int recvcounts[], MPI_Datatype dt, MPI_Op op,
                        MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPI_Reduce_scatter";
    if (!g_initialized || g_finalized) return err_return(comm, MPI_ERR_OTHER, fn);
    if (comm_index(comm) < 0) return err_return(comm, MPI_ERR_COMM, fn);
    const int n = comm == MPI_COMM_SELF ? 1 : mv2h_size();
    std::vector<size_t> rc_sz(n);
    size_t total = 0;
    for (int j = 0; j < n; ++j) {  // red_scat.c:1168-1171: the counts first
        if (recvcounts[j] < 0) return err_return(comm, MPI_ERR_COUNT, fn);
        rc_sz[j] = (size_t)recvcounts[j];
        total += rc_sz[j];
    }
    int rc = coll_checks(comm, 0, dt, op,
                         reduce_scatter_buf_checks(sendbuf, recvbuf, recvcounts[comm_rank_of(comm)], (long)total, dt));
    if (rc) return err_return(comm, rc, fn);
    if (total == 0) return MPI_SUCCESS;
    if (UserOp *u = user_op(op))
        if (comm != MPI_COMM_SELF)
            return err_return(comm, user_reduce_scatter(sendbuf, recvbuf, recvcounts, dt, u,
                                                        u->commute ? OPK_USER_COMM : OPK_USER_NONCOMM), fn);
    if (is_x87(dt) && comm != MPI_COMM_SELF && op_index(op) < OP_REPLACE) {
        UserOp x{ld_uop, 1, true};
        g_ld_op = op_index(op);
        return err_return(comm, user_reduce_scatter(sendbuf, recvbuf, recvcounts, dt, &x, OPK_BUILTIN), fn);
    }
    if (comm == MPI_COMM_SELF) {
        if (sendbuf != MPI_IN_PLACE)
            rc = mv2h_memcpy_dtod(recvbuf, sendbuf, dtype_span(dt, recvcounts[0]));
        return err_return(comm, rc, fn);
    }
    rc = mv2h_reduce_scatter(sendbuf, recvbuf, rc_sz.data(), dt, op, nullptr);
    return err_return(comm, rc, fn);
}
int MPI_Reduce_scatter(const void *sendbuf, void *recvbuf, const int recvcounts[], MPI_Datatype dt, MPI_Op op,
                       MPI_Comm comm) WEAK(MPI_Reduce_scatter);

int PMPI_Reduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount, MPI_Datatype dt, MPI_Op op,
                              MPI_Comm comm) {
    // MVAPICH2's MPIR_Reduce_scatter_block_MV2 never sizes the message (nbytes stays 0,
    // red_scat_block_osu.c:320-372), so the default table's first entry runs: MPICH's
    // MPIR_Reduce_scatter_block (red_scat_block.c:305, :515: recursive halving below
    // MPIR_CVAR_REDSCAT_COMMUTATIVE_LONG_MSG_SIZE, pairwise from it) — the same
    // selection as MPI_Ireduce_scatter_block's schedule
    const int n = comm == MPI_COMM_SELF ? 1 : mv2h_size();
    std::vector<int> counts(n, recvcount);
    const bool set = nbc_kind() == NBC_NONE;
    if (set) nbc_set(NBC_IREDUCE_SCATTER_BLOCK);
    const int rc = PMPI_Reduce_scatter(sendbuf, recvbuf, counts.data(), dt, op, comm);
    if (set) nbc_set(NBC_NONE);
    return rc;
}
int MPI_Reduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount, MPI_Datatype dt, MPI_Op op,
                             MPI_Comm comm) WEAK(MPI_Reduce_scatter_block);

// Allgather with a non-contiguous type on either side: pack this rank's
// contribution on the device, gather the packed bytes, and unpack all n
// blocks with one launch (block i of recvbuf starts i*recvcount extents in,
// so the n blocks are n*recvcount consecutive elements of recvtype).  The
// reference stages derived types through Localcopy / segment pack
// (allgather_osu.c:2426, helper_fns.h:62-250).
static int allgather_derived(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf, int recvcount,
                             MPI_Datatype recvtype, MPI_Comm comm) {
    const long rsize = dtype_size(recvtype), rext = dtype_extent(recvtype);
    const long psize = rsize * recvcount;
    if (sendbuf != MPI_IN_PLACE && dtype_size(sendtype) * sendcount != psize) return MPI_ERR_TRUNCATE;
    if (psize == 0) return MPI_SUCCESS;
    const int n = comm == MPI_COMM_SELF ? 1 : mv2h_size(), me = comm == MPI_COMM_SELF ? 0 : mv2h_rank();
    void *mine = pool_get((size_t)psize), *all = mine ? pool_get((size_t)psize * n) : nullptr;
    if (!all) {
        if (mine) pool_put(mine);
        return MPI_ERR_NO_MEM;
    }
    int pos = 0, rc;
    if (sendbuf == MPI_IN_PLACE)
        rc = PMPI_Pack((const char *)recvbuf + (long)me * recvcount * rext, recvcount, recvtype, mine, (int)psize, &pos,
                       comm);
    else
        rc = PMPI_Pack(sendbuf, sendcount, sendtype, mine, (int)psize, &pos, comm);
    if (!rc) rc = n > 1 ? mv2h_allgather(mine, all, (size_t)psize, nullptr) : mv2h_memcpy_dtod(all, mine, (size_t)psize);
    pos = 0;
    if (!rc) rc = PMPI_Unpack(all, (int)(psize * n), &pos, recvbuf, recvcount * n, recvtype, comm);
    pool_put(mine);
    pool_put(all);
    return rc;
}

int PMPI_Allgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf, int recvcount,
                   MPI_Datatype recvtype, MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPI_Allgather";
    if (!g_initialized) return err_return(comm, MPI_ERR_OTHER, fn);
    if (comm_index(comm) < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_COMM, fn);
    if (allgather_alias(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, comm_rank_of(comm)))
        return err_return(comm, MPI_ERR_BUFFER, fn);
    if (recvcount < 0 || (sendbuf != MPI_IN_PLACE && sendcount < 0)) return err_return(comm, MPI_ERR_COUNT, fn);
    if (!dtype_valid(recvtype) || (sendbuf != MPI_IN_PLACE && !dtype_valid(sendtype)))
        return err_return(comm, MPI_ERR_TYPE, fn);
    if (!dtype_committed(recvtype) || (sendbuf != MPI_IN_PLACE && !dtype_committed(sendtype)))
        return err_return(comm, MPI_ERR_TYPE, fn);
    if (const int rc = allgather_buf_checks(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype))
        return err_return(comm, rc, fn);
    if (!dtype_is_contiguous(recvtype) || (sendbuf != MPI_IN_PLACE && !dtype_is_contiguous(sendtype)))
        return err_return(comm, allgather_derived(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, comm), fn);
    const size_t rbytes = (size_t)dtype_span(recvtype, recvcount);
    if (sendbuf != MPI_IN_PLACE && (size_t)dtype_span(sendtype, sendcount) != rbytes)
        return err_return(comm, MPI_ERR_TRUNCATE, fn);
    if (rbytes == 0) return MPI_SUCCESS;
    if (comm == MPI_COMM_SELF) {
        int rc = sendbuf == MPI_IN_PLACE ? 0 : mv2h_memcpy_dtod(recvbuf, sendbuf, rbytes);
        return err_return(comm, rc, fn);
    }
    return err_return(comm, mv2h_allgather(sendbuf, recvbuf, rbytes, nullptr), fn);
}
int MPI_Allgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf, int recvcount,
                  MPI_Datatype recvtype, MPI_Comm comm) WEAK(MPI_Allgather);

int PMPI_Bcast(void *buffer, int count, MPI_Datatype dt, int root, MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPI_Bcast";
    if (!g_initialized) return err_return(comm, MPI_ERR_OTHER, fn);
    if (comm_index(comm) < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_COMM, fn);
    if (count < 0) return err_return(comm, MPI_ERR_COUNT, fn);
    if (!dtype_valid(dt)) return err_return(comm, MPI_ERR_TYPE, fn);
    const int size = comm == MPI_COMM_SELF ? 1 : mv2h_size();
    if (root < 0 || root >= size) return err_return(comm, MPI_ERR_ROOT, fn);
    if (!dtype_committed(dt)) return err_return(comm, MPI_ERR_TYPE, fn);
    if (inplace_buf(buffer, count) || null_userbuf(buffer, count, dt)) return err_return(comm, MPI_ERR_BUFFER, fn);  // bcast.c:1581-1582
    if (count == 0 || size == 1) return MPI_SUCCESS;
    if (dtype_is_contiguous(dt)) return err_return(comm, mv2h_bcast(buffer, (size_t)dtype_span(dt, count), root, nullptr), fn);
    // derived (non-contiguous) type: pack on device at the root, broadcast the
    // packed bytes, unpack on device everywhere else
    int psize = 0;
    PMPI_Pack_size(count, dt, comm, &psize);
    void *packed = pool_get((size_t)psize);
    if (!packed) return err_return(comm, MPI_ERR_NO_MEM, fn);
    int pos = 0, rc = MPI_SUCCESS;
    if (mv2h_rank() == root) rc = PMPI_Pack(buffer, count, dt, packed, psize, &pos, comm);
    if (!rc) rc = mv2h_bcast(packed, (size_t)psize, root, nullptr);
    pos = 0;
    if (!rc && mv2h_rank() != root) rc = PMPI_Unpack(packed, psize, &pos, buffer, count, dt, comm);
    pool_put(packed);
    return err_return(comm, rc, fn);
}
int MPI_Bcast(void *buffer, int count, MPI_Datatype dt, int root, MPI_Comm comm) WEAK(MPI_Bcast);

// ---------------------------------------------------------------------------
// Stream-ordered collectives (extension; mv2h.h *_enqueue): argument checks of the blocking
// calls, then the same algorithms launched on the caller's HIP stream without waiting.
// Calls the host would have to finish after the kernel — user ops, x87 types, derived
// types, host buffers — are refused with MPI_ERR_ARG / MPI_ERR_TYPE instead of blocking.
// ---------------------------------------------------------------------------
static int enqueue_arg_checks(MPI_Datatype dt, MPI_Op op, void *stream) {
    if (!stream) return MPI_ERR_ARG;
    if (user_op(op)) return MPI_ERR_ARG;
    if (is_x87(dt) || !dtype_is_contiguous(dt)) return MPI_ERR_TYPE;
    return MPI_SUCCESS;
}

int PMPIX_Allreduce_enqueue(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, MPI_Comm comm,
                            void *stream) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPIX_Allreduce_enqueue";
    int rc = coll_checks(comm, count, dt, op, allreduce_buf_checks(sendbuf, recvbuf, count, dt));
    if (!rc) rc = enqueue_arg_checks(dt, op, stream);
    if (rc) return err_return(comm, rc, fn);
    if (count == 0) return MPI_SUCCESS;
    if (comm == MPI_COMM_SELF) {  // a stream-ordered copy
        if (sendbuf == MPI_IN_PLACE || sendbuf == recvbuf) return MPI_SUCCESS;
        if (!is_dev(sendbuf) || !is_dev(recvbuf)) return err_return(comm, MPI_ERR_ARG, fn);
        return err_return(comm, mv2h_copy_enqueue(recvbuf, sendbuf, (size_t)dtype_span(dt, count), stream), fn);
    }
    return err_return(comm, mv2h_allreduce_enqueue(sendbuf, recvbuf, (size_t)count, dt, op, stream), fn);
}
int MPIX_Allreduce_enqueue(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, MPI_Comm comm,
                           void *stream) WEAK(MPIX_Allreduce_enqueue);

int PMPIX_Reduce_enqueue(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, int root,
                         MPI_Comm comm, void *stream) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPIX_Reduce_enqueue";
    if (!g_initialized || g_finalized) return err_return(comm, MPI_ERR_OTHER, fn);
    if (comm_index(comm) < 0) return err_return(comm, MPI_ERR_COMM, fn);
    const int size = comm == MPI_COMM_SELF ? 1 : mv2h_size();
    if (root < 0 || root >= size) return err_return(comm, MPI_ERR_ROOT, fn);
    int rc = coll_checks(comm, count, dt, op, reduce_buf_checks(sendbuf, recvbuf, count, dt, comm_rank_of(comm) == root));
    if (!rc) rc = enqueue_arg_checks(dt, op, stream);
    if (rc) return err_return(comm, rc, fn);
    if (count == 0) return MPI_SUCCESS;
    if (comm == MPI_COMM_SELF) return PMPIX_Allreduce_enqueue(sendbuf, recvbuf, count, dt, op, comm, stream);
    return err_return(comm, mv2h_reduce_enqueue(sendbuf, recvbuf, (size_t)count, dt, op, root, stream), fn);
}
int MPIX_Reduce_enqueue(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, int root,
                        MPI_Comm comm, void *stream) WEAK(MPIX_Reduce_enqueue);

int PMPIX_Reduce_scatter_enqueue(const void *sendbuf, void *recvbuf, const int recvcounts[], MPI_Datatype dt, MPI_Op op,
                                 MPI_Comm comm, void *stream) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPIX_Reduce_scatter_enqueue";
    if (!g_initialized || g_finalized) return err_return(comm, MPI_ERR_OTHER, fn);
    if (comm_index(comm) < 0) return err_return(comm, MPI_ERR_COMM, fn);
    if (!recvcounts) return err_return(comm, MPI_ERR_ARG, fn);
    const int n = comm == MPI_COMM_SELF ? 1 : mv2h_size();
    std::vector<size_t> rc_sz(n);
    size_t total = 0;
    for (int j = 0; j < n; ++j) {
        if (recvcounts[j] < 0) return err_return(comm, MPI_ERR_COUNT, fn);
        rc_sz[j] = (size_t)recvcounts[j];
        total += rc_sz[j];
    }
    int rc = coll_checks(comm, 0, dt, op,
                         reduce_scatter_buf_checks(sendbuf, recvbuf, recvcounts[comm_rank_of(comm)], (long)total, dt));
    if (!rc) rc = enqueue_arg_checks(dt, op, stream);
    if (rc) return err_return(comm, rc, fn);
    if (total == 0) return MPI_SUCCESS;
    if (comm == MPI_COMM_SELF) return PMPIX_Allreduce_enqueue(sendbuf, recvbuf, recvcounts[0], dt, op, comm, stream);
    return err_return(comm, mv2h_reduce_scatter_enqueue(sendbuf, recvbuf, rc_sz.data(), dt, op, stream), fn);
}
int MPIX_Reduce_scatter_enqueue(const void *sendbuf, void *recvbuf, const int recvcounts[], MPI_Datatype dt, MPI_Op op,
                                MPI_Comm comm, void *stream) WEAK(MPIX_Reduce_scatter_enqueue);

int PMPIX_Allgather_enqueue(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf, int recvcount,
                            MPI_Datatype recvtype, MPI_Comm comm, void *stream) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPIX_Allgather_enqueue";
    if (!g_initialized) return err_return(comm, MPI_ERR_OTHER, fn);
    if (comm_index(comm) < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_COMM, fn);
    if (!stream) return err_return(comm, MPI_ERR_ARG, fn);
    if (allgather_alias(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, comm_rank_of(comm)))
        return err_return(comm, MPI_ERR_BUFFER, fn);
    if (recvcount < 0 || (sendbuf != MPI_IN_PLACE && sendcount < 0)) return err_return(comm, MPI_ERR_COUNT, fn);
    if (!dtype_valid(recvtype) || (sendbuf != MPI_IN_PLACE && !dtype_valid(sendtype)))
        return err_return(comm, MPI_ERR_TYPE, fn);
    if (!dtype_committed(recvtype) || (sendbuf != MPI_IN_PLACE && !dtype_committed(sendtype)))
        return err_return(comm, MPI_ERR_TYPE, fn);
    if (const int rc = allgather_buf_checks(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype))
        return err_return(comm, rc, fn);
    if (!dtype_is_contiguous(recvtype) || (sendbuf != MPI_IN_PLACE && !dtype_is_contiguous(sendtype)))
        return err_return(comm, MPI_ERR_TYPE, fn);
    const size_t rbytes = (size_t)dtype_span(recvtype, recvcount);
    if (sendbuf != MPI_IN_PLACE && (size_t)dtype_span(sendtype, sendcount) != rbytes)
        return err_return(comm, MPI_ERR_TRUNCATE, fn);
    if (rbytes == 0) return MPI_SUCCESS;
    if (comm == MPI_COMM_SELF) {
        if (sendbuf == MPI_IN_PLACE || sendbuf == recvbuf) return MPI_SUCCESS;
        if (!is_dev(sendbuf) || !is_dev(recvbuf)) return err_return(comm, MPI_ERR_ARG, fn);
        return err_return(comm, mv2h_copy_enqueue(recvbuf, sendbuf, rbytes, stream), fn);
    }
    return err_return(comm, mv2h_allgather_enqueue(sendbuf, recvbuf, rbytes, stream), fn);
}
int MPIX_Allgather_enqueue(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf, int recvcount,
                           MPI_Datatype recvtype, MPI_Comm comm, void *stream) WEAK(MPIX_Allgather_enqueue);

int PMPIX_Bcast_enqueue(void *buffer, int count, MPI_Datatype dt, int root, MPI_Comm comm, void *stream) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    const char *fn = "MPIX_Bcast_enqueue";
    if (!g_initialized) return err_return(comm, MPI_ERR_OTHER, fn);
    if (comm_index(comm) < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_COMM, fn);
    if (!stream) return err_return(comm, MPI_ERR_ARG, fn);
    if (count < 0) return err_return(comm, MPI_ERR_COUNT, fn);
    if (!dtype_valid(dt) || !dtype_committed(dt)) return err_return(comm, MPI_ERR_TYPE, fn);
    if (!dtype_is_contiguous(dt)) return err_return(comm, MPI_ERR_TYPE, fn);
    const int size = comm == MPI_COMM_SELF ? 1 : mv2h_size();
    if (root < 0 || root >= size) return err_return(comm, MPI_ERR_ROOT, fn);
    if (inplace_buf(buffer, count) || null_userbuf(buffer, count, dt)) return err_return(comm, MPI_ERR_BUFFER, fn);
    if (count == 0 || size == 1) return MPI_SUCCESS;
    return err_return(comm, mv2h_bcast_enqueue(buffer, (size_t)dtype_span(dt, count), root, stream), fn);
}
int MPIX_Bcast_enqueue(void *buffer, int count, MPI_Datatype dt, int root, MPI_Comm comm, void *stream)
    WEAK(MPIX_Bcast_enqueue);

int PMPIX_Enqueue_check(MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    if (comm_index(comm) < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_COMM, "MPIX_Enqueue_check");
    return err_return(comm, mv2h_enqueue_check(), "MPIX_Enqueue_check");
}
int MPIX_Enqueue_check(MPI_Comm comm) WEAK(MPIX_Enqueue_check);

}  // extern "C"

// ---------------------------------------------------------------- requests
// One table for nonblocking collectives (completion-word tickets, mv2h_defer_*)
// and point-to-point requests (mv2h_isend / mv2h_irecv ids).  Handles are
// kReqBase | slot; MPI_REQUEST_NULL is MPICH's 0x2c000000.
namespace {
enum ReqKind { RQ_COLL = 1, RQ_P2P = 2, RQ_DONE = 3 };
struct MReq {
    int kind = 0;
    unsigned long long id = 0;
    bool live = false;
    bool is_recv = false;
    int src = MPI_ANY_SOURCE, tag = MPI_ANY_TAG;  // RQ_DONE status
    // derived-type staging: send keeps its packed copy, receive unpacks at completion
    void *tmp = nullptr;
    bool tmp_dev = false;
    int tmp_bytes = 0;
    void *ubuf = nullptr;
    MPI_Datatype dt = MPI_DATATYPE_NULL;
    int err = MPI_SUCCESS;  // a collective's error found by a peek (MPI_Testall), reported at completion
};
std::vector<MReq> g_mreqs;
constexpr MPI_Request kReqBase = (MPI_Request)0xac000000;

MPI_Request req_new(const MReq &r) {
    for (size_t i = 0; i < g_mreqs.size(); ++i)
        if (!g_mreqs[i].live) {
            g_mreqs[i] = r;
            g_mreqs[i].live = true;
            return kReqBase | (MPI_Request)i;
        }
    g_mreqs.push_back(r);
    g_mreqs.back().live = true;
    return kReqBase | (MPI_Request)(g_mreqs.size() - 1);
}

MReq *req_get(MPI_Request h) {
    if ((h & 0xfc000000) != (kReqBase & 0xfc000000)) return nullptr;
    const size_t i = (size_t)(h & 0x03ffffff);
    return i < g_mreqs.size() && g_mreqs[i].live ? &g_mreqs[i] : nullptr;
}

void status_set(MPI_Status *st, int src, int tag, size_t bytes, int err) {
    if (!st || st == MPI_STATUS_IGNORE) return;
    st->MPI_SOURCE = src;
    st->MPI_TAG = tag;
    st->MPI_ERROR = err;
    st->count_lo = (int)(bytes & 0xffffffffu);
    st->count_hi_and_cancelled = (int)((bytes >> 32) << 1);
}

void tmp_free(MReq &r) {
    if (!r.tmp) return;
    if (r.tmp_dev) pool_put(r.tmp);
    else free(r.tmp);
    r.tmp = nullptr;
}

// finish a request whose underlying operation completed (rc = its error class)
int req_finish(MReq &r, int rc, int src, int tag, size_t bytes, MPI_Status *st) {
    if (r.kind == RQ_P2P && r.is_recv && r.tmp && (rc == MPI_SUCCESS || rc == MPI_ERR_TRUNCATE)) {
        const long tsz = dtype_size(r.dt);
        const int nel = tsz > 0 ? (int)(bytes / (size_t)tsz) : 0;
        int pos = 0;
        const int urc = PMPI_Unpack(r.tmp, (int)bytes, &pos, r.ubuf, nel, r.dt, MPI_COMM_WORLD);
        if (rc == MPI_SUCCESS) rc = urc;
    }
    tmp_free(r);
    if (r.kind == RQ_COLL) status_set(st, MPI_ANY_SOURCE, MPI_ANY_TAG, 0, rc);
    else if (r.kind == RQ_DONE) status_set(st, r.src, r.tag, 0, rc);
    else if (r.is_recv) status_set(st, src, tag, bytes, rc);
    else status_set(st, MPI_ANY_SOURCE, MPI_ANY_TAG, 0, rc);
    r.live = false;
    return rc;
}

int req_wait(MReq &r, MPI_Status *st) {
    int src = MPI_ANY_SOURCE, tag = MPI_ANY_TAG, rc = MPI_SUCCESS;
    size_t bytes = 0;
    if (r.kind == RQ_COLL) rc = r.err ? r.err : mv2h_wait_ticket(r.id);
    else if (r.kind == RQ_P2P) rc = mv2h_p2p_wait(r.id, &src, &tag, &bytes);
    return req_finish(r, rc, src, tag, bytes, st);
}

int req_test(MReq &r, int *flag, MPI_Status *st) {
    int src = MPI_ANY_SOURCE, tag = MPI_ANY_TAG, rc = MPI_SUCCESS, done = 1;
    size_t bytes = 0;
    if (r.kind == RQ_COLL) rc = r.err ? r.err : mv2h_test_ticket(r.id, &done);
    else if (r.kind == RQ_P2P) rc = mv2h_p2p_test(r.id, &done, &src, &tag, &bytes);
    *flag = done;
    if (!done && rc == MPI_SUCCESS) return MPI_SUCCESS;
    *flag = 1;
    return req_finish(r, rc, src, tag, bytes, st);
}

// nonblocking collective = the blocking implementation initiated with
// deferred completion (the kernel is enqueued, the ticket waits later)
template <class F>
int start_coll(MPI_Request *request, const char *fn, F &&call, int nbc = MV2H_NBC_NONE) {
    if (!request) return err_return(MPI_COMM_WORLD, MPI_ERR_ARG, fn);
    mv2h_defer_begin();
    mv2h_nbc_begin(nbc);  // the nonblocking selection and reduction order (runtime/orders.h)
    const int rc = call();
    mv2h_nbc_end();
    unsigned long long t = 0;
    mv2h_defer_end(&t);
    if (rc) return rc;  // already passed through the error handler
    MReq r;
    r.kind = RQ_COLL;
    r.id = t;
    *request = req_new(r);
    return MPI_SUCCESS;
}

int p2p_checks(MPI_Comm comm, int count, MPI_Datatype dt, int tag, bool recv) {
    if (!g_initialized) return MPI_ERR_OTHER;
    if (comm != MPI_COMM_WORLD) return comm_index(comm) < 0 ? MPI_ERR_COMM : MPI_ERR_UNSUPPORTED_OPERATION;
    if (count < 0) return MPI_ERR_COUNT;
    if (!dtype_valid(dt) || !dtype_committed(dt)) return MPI_ERR_TYPE;
    if (recv ? (tag < 0 && tag != MPI_ANY_TAG) : tag < 0) return MPI_ERR_TAG;
    return MPI_SUCCESS;
}

int isend_impl(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Request *request) {
    MReq r;
    if (dest == MPI_PROC_NULL) {
        r.kind = RQ_DONE;
        r.src = MPI_PROC_NULL;
        *request = req_new(r);
        return MPI_SUCCESS;
    }
    if (dest < 0 || dest >= world().gsize) return MPI_ERR_RANK;
    r.kind = RQ_P2P;
    const void *src = buf;
    size_t bytes = (size_t)dtype_span(dt, count);
    if (!dtype_is_contiguous(dt)) {  // device (or host) pack first, the packed copy travels
        int psize = 0, pos = 0;
        PMPI_Pack_size(count, dt, MPI_COMM_WORLD, &psize);
        r.tmp_dev = is_dev(buf);
        if (r.tmp_dev) {
            if (!(r.tmp = pool_get((size_t)psize))) return MPI_ERR_NO_MEM;
        } else if (!(r.tmp = malloc((size_t)psize + 1))) {
            return MPI_ERR_NO_MEM;
        }
        const int rc = PMPI_Pack(buf, count, dt, r.tmp, psize, &pos, MPI_COMM_WORLD);
        if (rc) {
            tmp_free(r);
            return rc;
        }
        src = r.tmp;
        bytes = (size_t)pos;
    }
    const int rc = mv2h_isend(src, bytes, dest, tag, &r.id);
    if (rc) {
        tmp_free(r);
        return rc;
    }
    *request = req_new(r);
    return MPI_SUCCESS;
}

int irecv_impl(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Request *request) {
    MReq r;
    r.is_recv = true;
    if (source == MPI_PROC_NULL) {
        r.kind = RQ_DONE;
        r.src = MPI_PROC_NULL;
        *request = req_new(r);
        return MPI_SUCCESS;
    }
    if (source != MPI_ANY_SOURCE && (source < 0 || source >= world().gsize)) return MPI_ERR_RANK;
    r.kind = RQ_P2P;
    void *dst = buf;
    size_t cap = (size_t)dtype_span(dt, count);
    if (!dtype_is_contiguous(dt)) {  // receive packed, unpack at completion
        int psize = 0;
        PMPI_Pack_size(count, dt, MPI_COMM_WORLD, &psize);
        r.tmp_dev = is_dev(buf);
        if (r.tmp_dev) {
            if (!(r.tmp = pool_get((size_t)psize))) return MPI_ERR_NO_MEM;
        } else if (!(r.tmp = malloc((size_t)psize + 1))) {
            return MPI_ERR_NO_MEM;
        }
        r.ubuf = buf;
        r.dt = dt;
        dst = r.tmp;
        cap = (size_t)psize;
    }
    const int rc = mv2h_irecv(dst, cap, source, tag, &r.id);
    if (rc) {
        tmp_free(r);
        return rc;
    }
    *request = req_new(r);
    return MPI_SUCCESS;
}

}  // namespace

extern "C" {

int PMPI_Iallreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, MPI_Comm comm,
                    MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    return start_coll(
        request, "MPI_Iallreduce", [&] { return PMPI_Allreduce(sendbuf, recvbuf, count, dt, op, comm); },
        MV2H_NBC_IALLREDUCE);
}
int MPI_Iallreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, MPI_Comm comm,
                   MPI_Request *request) WEAK(MPI_Iallreduce);

int PMPI_Ireduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, int root, MPI_Comm comm,
                 MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    return start_coll(
        request, "MPI_Ireduce", [&] { return PMPI_Reduce(sendbuf, recvbuf, count, dt, op, root, comm); },
        MV2H_NBC_IREDUCE);
}
int MPI_Ireduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op, int root, MPI_Comm comm,
                MPI_Request *request) WEAK(MPI_Ireduce);

int PMPI_Ireduce_scatter(const void *sendbuf, void *recvbuf, const int recvcounts[], MPI_Datatype dt, MPI_Op op,
                         MPI_Comm comm, MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    return start_coll(
        request, "MPI_Ireduce_scatter", [&] { return PMPI_Reduce_scatter(sendbuf, recvbuf, recvcounts, dt, op, comm); },
        MV2H_NBC_IREDUCE_SCATTER);
}
int MPI_Ireduce_scatter(const void *sendbuf, void *recvbuf, const int recvcounts[], MPI_Datatype dt, MPI_Op op,
                        MPI_Comm comm, MPI_Request *request) WEAK(MPI_Ireduce_scatter);

int PMPI_Ireduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount, MPI_Datatype dt, MPI_Op op,
                               MPI_Comm comm, MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    return start_coll(
        request, "MPI_Ireduce_scatter_block",
        [&] { return PMPI_Reduce_scatter_block(sendbuf, recvbuf, recvcount, dt, op, comm); },
        MV2H_NBC_IREDUCE_SCATTER_BLOCK);
}
int MPI_Ireduce_scatter_block(const void *sendbuf, void *recvbuf, int recvcount, MPI_Datatype dt, MPI_Op op,
                              MPI_Comm comm, MPI_Request *request) WEAK(MPI_Ireduce_scatter_block);

int PMPI_Iallgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf, int recvcount,
                    MPI_Datatype recvtype, MPI_Comm comm, MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    return start_coll(request, "MPI_Iallgather", [&] {
        return PMPI_Allgather(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, comm);
    });
}
int MPI_Iallgather(const void *sendbuf, int sendcount, MPI_Datatype sendtype, void *recvbuf, int recvcount,
                   MPI_Datatype recvtype, MPI_Comm comm, MPI_Request *request) WEAK(MPI_Iallgather);

int PMPI_Ibcast(void *buffer, int count, MPI_Datatype dt, int root, MPI_Comm comm, MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    return start_coll(request, "MPI_Ibcast", [&] { return PMPI_Bcast(buffer, count, dt, root, comm); });
}
int MPI_Ibcast(void *buffer, int count, MPI_Datatype dt, int root, MPI_Comm comm, MPI_Request *request)
    WEAK(MPI_Ibcast);

int PMPI_Ibarrier(MPI_Comm comm, MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    return start_coll(request, "MPI_Ibarrier", [&] { return PMPI_Barrier(comm); });
}
int MPI_Ibarrier(MPI_Comm comm, MPI_Request *request) WEAK(MPI_Ibarrier);

int PMPI_Wait(MPI_Request *request, MPI_Status *status) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    if (!request) return err_return(MPI_COMM_WORLD, MPI_ERR_ARG, "MPI_Wait");
    if (*request == MPI_REQUEST_NULL) {
        status_set(status, MPI_ANY_SOURCE, MPI_ANY_TAG, 0, MPI_SUCCESS);
        return MPI_SUCCESS;
    }
    MReq *r = req_get(*request);
    if (!r) return err_return(MPI_COMM_WORLD, MPI_ERR_REQUEST, "MPI_Wait");
    const int rc = req_wait(*r, status);
    *request = MPI_REQUEST_NULL;
    return err_return(MPI_COMM_WORLD, rc, "MPI_Wait");
}
int MPI_Wait(MPI_Request *request, MPI_Status *status) WEAK(MPI_Wait);

int PMPI_Test(MPI_Request *request, int *flag, MPI_Status *status) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    if (!request || !flag) return err_return(MPI_COMM_WORLD, MPI_ERR_ARG, "MPI_Test");
    if (*request == MPI_REQUEST_NULL) {
        *flag = 1;
        status_set(status, MPI_ANY_SOURCE, MPI_ANY_TAG, 0, MPI_SUCCESS);
        return MPI_SUCCESS;
    }
    MReq *r = req_get(*request);
    if (!r) return err_return(MPI_COMM_WORLD, MPI_ERR_REQUEST, "MPI_Test");
    const int rc = req_test(*r, flag, status);
    if (*flag) *request = MPI_REQUEST_NULL;
    return err_return(MPI_COMM_WORLD, rc, "MPI_Test");
}
int MPI_Test(MPI_Request *request, int *flag, MPI_Status *status) WEAK(MPI_Test);

int PMPI_Waitall(int count, MPI_Request requests[], MPI_Status statuses[]) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    if (count < 0 || (count && !requests)) return err_return(MPI_COMM_WORLD, MPI_ERR_ARG, "MPI_Waitall");
    // progress every request together (a receive may need a send of this rank to move)
    int rc_all = MPI_SUCCESS;
    for (;;) {
        bool pending = false;
        for (int i = 0; i < count; ++i) {
            if (requests[i] == MPI_REQUEST_NULL) continue;
            MReq *r = req_get(requests[i]);
            MPI_Status *st = (!statuses || statuses == MPI_STATUSES_IGNORE) ? MPI_STATUS_IGNORE : &statuses[i];
            if (!r) {
                status_set(st, MPI_ANY_SOURCE, MPI_ANY_TAG, 0, MPI_ERR_REQUEST);
                rc_all = MPI_ERR_IN_STATUS;
                requests[i] = MPI_REQUEST_NULL;
                continue;
            }
            int flag = 0;
            const int rc = req_test(*r, &flag, st);
            if (flag) {
                requests[i] = MPI_REQUEST_NULL;
                if (rc) rc_all = MPI_ERR_IN_STATUS;
            } else {
                pending = true;
            }
        }
        if (!pending) break;
        sched_yield();
    }
    return err_return(MPI_COMM_WORLD, rc_all, "MPI_Waitall");
}
int MPI_Waitall(int count, MPI_Request requests[], MPI_Status statuses[]) WEAK(MPI_Waitall);

int PMPI_Testall(int count, MPI_Request requests[], int *flag, MPI_Status statuses[]) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    if (count < 0 || !flag || (count && !requests)) return err_return(MPI_COMM_WORLD, MPI_ERR_ARG, "MPI_Testall");
    // MPI-3.1 §3.7.5: flag = true only if all requests have completed, and then all of them
    // are completed (deallocated, statuses set); otherwise no request is modified.  First a
    // peek (progress without completing), then completion of all of them.
    for (int i = 0; i < count; ++i) {
        if (requests[i] == MPI_REQUEST_NULL) continue;
        MReq *r = req_get(requests[i]);
        if (!r) continue;  // reported below
        int d = 1;
        if (r->kind == RQ_COLL) {
            const int rc = mv2h_test_ticket(r->id, &d);  // reads the completion word only
            if (rc) r->err = rc, d = 1;                  // a failed collective has completed
        } else if (r->kind == RQ_P2P && mv2h_p2p_peek(r->id, &d)) {
            d = 1;  // the request's own test reports the error
        }
        if (!d) {
            *flag = 0;
            return MPI_SUCCESS;
        }
    }
    int rc_all = MPI_SUCCESS;
    for (int i = 0; i < count; ++i) {
        if (requests[i] == MPI_REQUEST_NULL) continue;
        MReq *r = req_get(requests[i]);
        MPI_Status *st = (!statuses || statuses == MPI_STATUSES_IGNORE) ? MPI_STATUS_IGNORE : &statuses[i];
        if (!r) {
            status_set(st, MPI_ANY_SOURCE, MPI_ANY_TAG, 0, MPI_ERR_REQUEST);
            requests[i] = MPI_REQUEST_NULL;
            rc_all = MPI_ERR_IN_STATUS;
            continue;
        }
        const int rc = req_wait(*r, st);  // complete: returns at once
        requests[i] = MPI_REQUEST_NULL;
        if (rc) rc_all = MPI_ERR_IN_STATUS;
    }
    *flag = 1;
    return err_return(MPI_COMM_WORLD, rc_all, "MPI_Testall");
}
int MPI_Testall(int count, MPI_Request requests[], int *flag, MPI_Status statuses[]) WEAK(MPI_Testall);

int PMPI_Request_free(MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    if (!request) return err_return(MPI_COMM_WORLD, MPI_ERR_ARG, "MPI_Request_free");
    MReq *r = req_get(*request);
    if (!r) return err_return(MPI_COMM_WORLD, MPI_ERR_REQUEST, "MPI_Request_free");
    // the operation still completes; this library waits for it here
    req_wait(*r, MPI_STATUS_IGNORE);
    *request = MPI_REQUEST_NULL;
    return MPI_SUCCESS;
}
int MPI_Request_free(MPI_Request *request) WEAK(MPI_Request_free);

// ---------------------------------------------------------------- point-to-point
int PMPI_Isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    int rc = p2p_checks(comm, count, dt, tag, false);
    if (!rc && !request) rc = MPI_ERR_ARG;
    if (!rc) rc = isend_impl(buf, count, dt, dest, tag, request);
    return err_return(comm, rc, "MPI_Isend");
}
int MPI_Isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *request)
    WEAK(MPI_Isend);

int PMPI_Irecv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Request *request) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    int rc = p2p_checks(comm, count, dt, tag, true);
    if (!rc && !request) rc = MPI_ERR_ARG;
    if (!rc) rc = irecv_impl(buf, count, dt, source, tag, request);
    return err_return(comm, rc, "MPI_Irecv");
}
int MPI_Irecv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Request *request)
    WEAK(MPI_Irecv);

int PMPI_Send(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    MPI_Request rq = MPI_REQUEST_NULL;
    int rc = p2p_checks(comm, count, dt, tag, false);
    if (!rc) rc = isend_impl(buf, count, dt, dest, tag, &rq);
    if (!rc) rc = req_wait(*req_get(rq), MPI_STATUS_IGNORE);
    return err_return(comm, rc, "MPI_Send");
}
int MPI_Send(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm) WEAK(MPI_Send);

int PMPI_Recv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Status *status) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    MPI_Request rq = MPI_REQUEST_NULL;
    int rc = p2p_checks(comm, count, dt, tag, true);
    if (!rc) rc = irecv_impl(buf, count, dt, source, tag, &rq);
    if (!rc) rc = req_wait(*req_get(rq), status);
    return err_return(comm, rc, "MPI_Recv");
}
int MPI_Recv(void *buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Status *status)
    WEAK(MPI_Recv);

int PMPI_Sendrecv(const void *sendbuf, int sendcount, MPI_Datatype sendtype, int dest, int sendtag, void *recvbuf,
                  int recvcount, MPI_Datatype recvtype, int source, int recvtag, MPI_Comm comm, MPI_Status *status) {
    std::lock_guard<std::recursive_mutex> lk(g_cs);
    MPI_Request rr = MPI_REQUEST_NULL, sr = MPI_REQUEST_NULL;
    int rc = p2p_checks(comm, recvcount, recvtype, recvtag, true);
    if (!rc) rc = p2p_checks(comm, sendcount, sendtype, sendtag, false);
    if (!rc) rc = irecv_impl(recvbuf, recvcount, recvtype, source, recvtag, &rr);
    if (!rc) rc = isend_impl(sendbuf, sendcount, sendtype, dest, sendtag, &sr);
    if (rc) return err_return(comm, rc, "MPI_Sendrecv");
    MPI_Request both[2] = {rr, sr};
    MPI_Status sts[2];
    rc = PMPI_Waitall(2, both, sts);
    if (status && status != MPI_STATUS_IGNORE) *status = sts[0];
    if (rc == MPI_ERR_IN_STATUS) rc = sts[0].MPI_ERROR ? sts[0].MPI_ERROR : sts[1].MPI_ERROR;
    return err_return(comm, rc, "MPI_Sendrecv");
}
int MPI_Sendrecv(const void *sendbuf, int sendcount, MPI_Datatype sendtype, int dest, int sendtag, void *recvbuf,
                 int recvcount, MPI_Datatype recvtype, int source, int recvtag, MPI_Comm comm, MPI_Status *status)
    WEAK(MPI_Sendrecv);

int PMPI_Get_count(const MPI_Status *status, MPI_Datatype dt, int *count) {
    if (!status || !count) return err_return(MPI_COMM_WORLD, MPI_ERR_ARG, "MPI_Get_count");
    const long tsz = dtype_size(dt);
    if (tsz < 0) return err_return(MPI_COMM_WORLD, MPI_ERR_TYPE, "MPI_Get_count");
    const unsigned long long bytes = (unsigned long long)(unsigned)status->count_lo |
                                     ((unsigned long long)((unsigned)status->count_hi_and_cancelled >> 1) << 32);
    if (tsz == 0) *count = 0;
    else *count = bytes % (unsigned long long)tsz ? MPI_UNDEFINED : (int)(bytes / (unsigned long long)tsz);
    return MPI_SUCCESS;
}
int MPI_Get_count(const MPI_Status *status, MPI_Datatype dt, int *count) WEAK(MPI_Get_count);

}  // extern "C"
