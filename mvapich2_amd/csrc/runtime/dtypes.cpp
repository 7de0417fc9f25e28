// dtypes.cpp — builtin datatype table (MPICH ABI, LP64).
// Handles: reference configure.ac:3475-3530 / 3707-3733 / 3878-4060;
// groups: oputil.h:274-372; pair sizes: mpid_type_create_pairtype.c.
#include <stddef.h>

#include "../common.h"

namespace mv2 {

static const DtypeInfo kTypes[] = {
    // C integer group (oputil.h:274-292)
    {0x4c000405, K_I32, 4, 4, G_CINT, "MPI_INT"},
    {0x4c000807, K_I64, 8, 8, G_CINT, "MPI_LONG"},
    {0x4c000203, K_I16, 2, 2, G_CINT, "MPI_SHORT"},
    {0x4c000204, K_U16, 2, 2, G_CINT, "MPI_UNSIGNED_SHORT"},
    {0x4c000406, K_U32, 4, 4, G_CINT, "MPI_UNSIGNED"},
    {0x4c000808, K_U64, 8, 8, G_CINT, "MPI_UNSIGNED_LONG"},
    {0x4c000809, K_I64, 8, 8, G_CINT, "MPI_LONG_LONG_INT"},
    {0x4c000819, K_U64, 8, 8, G_CINT, "MPI_UNSIGNED_LONG_LONG"},
    {0x4c000118, K_I8, 1, 1, G_CINT, "MPI_SIGNED_CHAR"},
    {0x4c000102, K_U8, 1, 1, G_CINT, "MPI_UNSIGNED_CHAR"},
    {0x4c000137, K_I8, 1, 1, G_CINT, "MPI_INT8_T"},
    {0x4c000238, K_I16, 2, 2, G_CINT, "MPI_INT16_T"},
    {0x4c000439, K_I32, 4, 4, G_CINT, "MPI_INT32_T"},
    {0x4c00083a, K_I64, 8, 8, G_CINT, "MPI_INT64_T"},
    {0x4c00013b, K_U8, 1, 1, G_CINT, "MPI_UINT8_T"},
    {0x4c00023c, K_U16, 2, 2, G_CINT, "MPI_UINT16_T"},
    {0x4c00043d, K_U32, 4, 4, G_CINT, "MPI_UINT32_T"},
    {0x4c00083e, K_U64, 8, 8, G_CINT, "MPI_UINT64_T"},
    // C integer extra (oputil.h:295-296): char is signed on x86-64
    {0x4c000101, K_I8, 1, 1, G_CINTX, "MPI_CHAR"},
    // Fortran integer group (oputil.h:299-303)
    {0x4c00041b, K_I32, 4, 4, G_FINT, "MPI_INTEGER"},
    {0x4c000843, K_I64, 8, 8, G_FINT, "MPI_AINT"},
    {0x4c000844, K_I64, 8, 8, G_FINT, "MPI_OFFSET"},
    {0x4c000845, K_I64, 8, 8, G_FINT, "MPI_COUNT"},
    // floating point (oputil.h:316-321)
    {0x4c00040a, K_F32, 4, 4, G_FP, "MPI_FLOAT"},
    {0x4c00080b, K_F64, 8, 8, G_FP, "MPI_DOUBLE"},
    {0x4c00041c, K_F32, 4, 4, G_FP, "MPI_REAL"},
    {0x4c00081f, K_F64, 8, 8, G_FP, "MPI_DOUBLE_PRECISION"},
    {0x4c00100c, K_LDOUBLE, 16, 16, G_FP, "MPI_LONG_DOUBLE"},
    // logical (oputil.h:331-334): LOGICAL via MPIR_TO/FROM_FLOG == int 0/1 logic
    {0x4c00041d, K_I32, 4, 4, G_LOGICAL, "MPI_LOGICAL"},
    {0x4c00013f, K_U8, 1, 1, G_LOGICAL, "MPI_C_BOOL"},
    // complex (oputil.h:338-349)
    {0x4c00081e, K_CF32_S, 8, 8, G_COMPLEX, "MPI_COMPLEX"},
    {0x4c000840, K_CF32_C99, 8, 8, G_COMPLEX, "MPI_C_FLOAT_COMPLEX"},
    {0x4c001041, K_CF64_C99, 16, 16, G_COMPLEX, "MPI_C_DOUBLE_COMPLEX"},
    {0x4c002042, K_LDOUBLE, 32, 32, G_COMPLEX, "MPI_C_LONG_DOUBLE_COMPLEX"},
    {0x4c001022, K_CF64_S, 16, 16, G_COMPLEX, "MPI_DOUBLE_COMPLEX"},
    // byte
    {0x4c00010d, K_U8, 1, 1, G_BYTE, "MPI_BYTE"},
    // MINLOC / MAXLOC pair types
    {0x4c000816, K_P_2INT, 8, 8, G_PAIR, "MPI_2INT"},
    {(int)0x8c000000, K_P_FLOATINT, 8, 8, G_PAIR, "MPI_FLOAT_INT"},
    {(int)0x8c000001, K_P_DOUBLEINT, 12, 16, G_PAIR, "MPI_DOUBLE_INT"},
    {(int)0x8c000002, K_P_LONGINT, 12, 16, G_PAIR, "MPI_LONG_INT"},
    {(int)0x8c000003, K_P_SHORTINT, 6, 8, G_PAIR, "MPI_SHORT_INT"},
    {(int)0x8c000004, K_LDOUBLE, 20, 32, G_PAIR, "MPI_LONG_DOUBLE_INT"},
    {0x4c000820, K_P_2INT, 8, 8, G_PAIR, "MPI_2INTEGER"},
    {0x4c000821, K_P_2F32, 8, 8, G_PAIR, "MPI_2REAL"},
    {0x4c001023, K_P_2F64, 16, 16, G_PAIR, "MPI_2DOUBLE_PRECISION"},
    // no reduction group
    {0x4c00040e, K_NONE, 4, 4, G_NONE, "MPI_WCHAR"},
    {0x4c00010f, K_NONE, 1, 1, G_NONE, "MPI_PACKED"},
};

const DtypeInfo *dtype_lookup(int handle) {
    for (const DtypeInfo &t : kTypes)
        if (t.handle == handle) return &t;
    return nullptr;
}

}  // namespace mv2
