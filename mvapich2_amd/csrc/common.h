// common.h — datatype / op tables shared by the host glue and the HIP kernels.
//
// Op index = (handle & 0xf) - 1 exactly as MPIR_OP_HDL_TO_FN (reference
// src/include/mpiimpl.h:4031) indexes MPIR_Op_table (allreduce.c:95-100).
// Type groups and op x group legality restate oputil.h:274-372 and the
// MPIR_*_check_dtype functions (opsum.c:95-123, opmax.c:70-95,
// opland.c:106-130, opband.c:57-80, opmaxloc.c:179-211 with the default
// Fortran-enabled build, opreplace.c:34-38).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace mv2 {

enum OpId : int {
    OP_MAX = 0, OP_MIN, OP_SUM, OP_PROD, OP_LAND, OP_BAND, OP_LOR, OP_BOR,
    OP_LXOR, OP_BXOR, OP_MINLOC, OP_MAXLOC, OP_REPLACE, OP_NO_OP, OP_COUNT
};

// Storage/arithmetic kind of one element.  Several MPI types share a kind
// (e.g. MPI_INT, MPI_INT32_T, MPI_INTEGER, MPI_LOGICAL -> K_I32).
enum Kind : int {
    K_I8 = 0, K_U8, K_I16, K_U16, K_I32, K_U32, K_I64, K_U64,
    K_F32, K_F64,
    K_CF32_C99,   // float _Complex     : C99 multiply (Annex G), componentwise add
    K_CF64_C99,   // double _Complex
    K_CF32_S,     // struct {float re,im}  (Fortran COMPLEX, opprod.c:43-54)
    K_CF64_S,     // struct {double re,im} (Fortran DOUBLE COMPLEX)
    K_P_2INT,     // {int value; int loc}        8/8
    K_P_FLOATINT, // {float value; int loc}      8/8
    K_P_LONGINT,  // {long value; int loc}       12/16
    K_P_SHORTINT, // {short value; int loc}      6/8
    K_P_DOUBLEINT,// {double value; int loc}     12/16
    K_P_2F32,     // MPI_2REAL   (flat float pair, loc compared as float)
    K_P_2F64,     // MPI_2DOUBLE_PRECISION
    K_LDOUBLE,    // x87 80-bit long double: not representable on gfx950 (unsupported)
    K_NONE,       // no arithmetic (MPI_WCHAR, MPI_PACKED)
    K_COUNT
};

enum Group : int {
    G_NONE = 0, G_CINT = 1, G_CINTX = 2, G_FINT = 4, G_FP = 8, G_LOGICAL = 16,
    G_COMPLEX = 32, G_BYTE = 64, G_PAIR = 128
};

struct DtypeInfo {
    int handle;
    int kind;
    int size;    // MPI_Type_size
    int extent;  // MPI_Type_get_extent
    int groups;
    const char *name;
};

// ---- op x group legality (host + device) ----
inline bool op_valid_for_groups(int op, int g) {
    switch (op) {
    case OP_SUM: case OP_PROD: return g & (G_CINT | G_CINTX | G_FINT | G_FP | G_COMPLEX);
    case OP_MAX: case OP_MIN: return g & (G_CINT | G_CINTX | G_FINT | G_FP);
    case OP_LAND: case OP_LOR: case OP_LXOR: return g & (G_CINT | G_CINTX | G_FINT | G_FP | G_LOGICAL);
    case OP_BAND: case OP_BOR: case OP_BXOR: return g & (G_CINT | G_CINTX | G_FINT | G_BYTE);
    case OP_MAXLOC: case OP_MINLOC: return g & G_PAIR;
    case OP_REPLACE: case OP_NO_OP: return true;
    default: return false;
    }
}

const DtypeInfo *dtype_lookup(int handle);  // builtin types only (host)

inline int op_index(int handle) { return (handle & 0xf) - 1; }
inline bool is_builtin_op(int handle) { return (handle & 0xfffffff0) == 0x58000000 && op_index(handle) >= 0 && op_index(handle) < OP_COUNT; }

// MPI error classes used by the HIP layer (mirror include/mpi.h)
enum { E_SUCCESS = 0, E_BUFFER = 1, E_COUNT = 2, E_TYPE = 3, E_TAG = 4, E_COMM = 5, E_RANK = 6, E_ROOT = 7, E_OP = 9,
       E_ARG = 12, E_TRUNCATE = 14, E_OTHER = 15, E_INTERN = 16, E_REQUEST = 19, E_NO_MEM = 34, E_UNSUPPORTED = 44 };

}  // namespace mv2
