"""MPICH-ABI handle values (mirror of include/mpi.h) for the Python bindings."""

MPI_SUCCESS = 0
MPI_ERR_BUFFER = 1
MPI_ERR_COUNT = 2
MPI_ERR_TYPE = 3
MPI_ERR_COMM = 5
MPI_ERR_ROOT = 7
MPI_ERR_OP = 9
MPI_ERR_ARG = 12
MPI_ERR_TRUNCATE = 14
MPI_ERR_OTHER = 15
MPI_ERR_INTERN = 16

MPI_COMM_WORLD = 0x44000000
MPI_COMM_SELF = 0x44000001
MPI_ERRORS_ARE_FATAL = 0x54000000
MPI_ERRORS_RETURN = 0x54000001
MPI_IN_PLACE = -1

OPS = {
    "MPI_MAX": 0x58000001, "MPI_MIN": 0x58000002, "MPI_SUM": 0x58000003,
    "MPI_PROD": 0x58000004, "MPI_LAND": 0x58000005, "MPI_BAND": 0x58000006,
    "MPI_LOR": 0x58000007, "MPI_BOR": 0x58000008, "MPI_LXOR": 0x58000009,
    "MPI_BXOR": 0x5800000A, "MPI_MINLOC": 0x5800000B, "MPI_MAXLOC": 0x5800000C,
    "MPI_REPLACE": 0x5800000D, "MPI_NO_OP": 0x5800000E,
}

# name -> (handle, numpy dtype description, size, extent)
# numpy descriptions: plain scalar codes, or structured dtypes for pair/complex types
TYPES = {
    "MPI_CHAR": (0x4C000101, "i1", 1, 1),
    "MPI_SIGNED_CHAR": (0x4C000118, "i1", 1, 1),
    "MPI_UNSIGNED_CHAR": (0x4C000102, "u1", 1, 1),
    "MPI_BYTE": (0x4C00010D, "u1", 1, 1),
    "MPI_SHORT": (0x4C000203, "i2", 2, 2),
    "MPI_UNSIGNED_SHORT": (0x4C000204, "u2", 2, 2),
    "MPI_INT": (0x4C000405, "i4", 4, 4),
    "MPI_UNSIGNED": (0x4C000406, "u4", 4, 4),
    "MPI_LONG": (0x4C000807, "i8", 8, 8),
    "MPI_UNSIGNED_LONG": (0x4C000808, "u8", 8, 8),
    "MPI_LONG_LONG": (0x4C000809, "i8", 8, 8),
    "MPI_UNSIGNED_LONG_LONG": (0x4C000819, "u8", 8, 8),
    "MPI_FLOAT": (0x4C00040A, "f4", 4, 4),
    "MPI_DOUBLE": (0x4C00080B, "f8", 8, 8),
    "MPI_LONG_DOUBLE": (0x4C00100C, "f16", 16, 16),
    "MPI_INT8_T": (0x4C000137, "i1", 1, 1),
    "MPI_INT16_T": (0x4C000238, "i2", 2, 2),
    "MPI_INT32_T": (0x4C000439, "i4", 4, 4),
    "MPI_INT64_T": (0x4C00083A, "i8", 8, 8),
    "MPI_UINT8_T": (0x4C00013B, "u1", 1, 1),
    "MPI_UINT16_T": (0x4C00023C, "u2", 2, 2),
    "MPI_UINT32_T": (0x4C00043D, "u4", 4, 4),
    "MPI_UINT64_T": (0x4C00083E, "u8", 8, 8),
    "MPI_C_BOOL": (0x4C00013F, "u1", 1, 1),
    "MPI_C_FLOAT_COMPLEX": (0x4C000840, "c8", 8, 8),
    "MPI_C_DOUBLE_COMPLEX": (0x4C001041, "c16", 16, 16),
    "MPI_AINT": (0x4C000843, "i8", 8, 8),
    "MPI_OFFSET": (0x4C000844, "i8", 8, 8),
    "MPI_COUNT": (0x4C000845, "i8", 8, 8),
    "MPI_INTEGER": (0x4C00041B, "i4", 4, 4),
    "MPI_REAL": (0x4C00041C, "f4", 4, 4),
    "MPI_LOGICAL": (0x4C00041D, "i4", 4, 4),
    "MPI_COMPLEX": (0x4C00081E, "c8", 8, 8),
    "MPI_DOUBLE_PRECISION": (0x4C00081F, "f8", 8, 8),
    "MPI_DOUBLE_COMPLEX": (0x4C001022, "c16", 16, 16),
    "MPI_2INT": (0x4C000816, [("value", "i4"), ("loc", "i4")], 8, 8),
    "MPI_FLOAT_INT": (0x8C000000, [("value", "f4"), ("loc", "i4")], 8, 8),
    "MPI_DOUBLE_INT": (0x8C000001, {"names": ["value", "loc"], "formats": ["f8", "i4"], "offsets": [0, 8], "itemsize": 16}, 12, 16),
    "MPI_LONG_INT": (0x8C000002, {"names": ["value", "loc"], "formats": ["i8", "i4"], "offsets": [0, 8], "itemsize": 16}, 12, 16),
    "MPI_SHORT_INT": (0x8C000003, {"names": ["value", "loc"], "formats": ["i2", "i4"], "offsets": [0, 4], "itemsize": 8}, 6, 8),
    "MPI_2INTEGER": (0x4C000820, [("value", "i4"), ("loc", "i4")], 8, 8),
    "MPI_2REAL": (0x4C000821, [("value", "f4"), ("loc", "f4")], 8, 8),
    "MPI_2DOUBLE_PRECISION": (0x4C001023, [("value", "f8"), ("loc", "f8")], 16, 16),
    "MPI_WCHAR": (0x4C00040E, "u4", 4, 4),
}

# MPI op x type-group legality (oputil.h:274-372 + MPIR_*_check_dtype)
GROUPS = {
    "C_INTEGER": ["MPI_INT", "MPI_LONG", "MPI_SHORT", "MPI_UNSIGNED_SHORT", "MPI_UNSIGNED",
                  "MPI_UNSIGNED_LONG", "MPI_LONG_LONG", "MPI_UNSIGNED_LONG_LONG", "MPI_SIGNED_CHAR",
                  "MPI_UNSIGNED_CHAR", "MPI_INT8_T", "MPI_INT16_T", "MPI_INT32_T", "MPI_INT64_T",
                  "MPI_UINT8_T", "MPI_UINT16_T", "MPI_UINT32_T", "MPI_UINT64_T"],
    "C_INTEGER_EXTRA": ["MPI_CHAR"],
    "FORTRAN_INTEGER": ["MPI_INTEGER", "MPI_AINT", "MPI_OFFSET", "MPI_COUNT"],
    "FLOATING_POINT": ["MPI_FLOAT", "MPI_DOUBLE", "MPI_REAL", "MPI_DOUBLE_PRECISION", "MPI_LONG_DOUBLE"],
    "LOGICAL": ["MPI_LOGICAL", "MPI_C_BOOL"],
    "COMPLEX": ["MPI_COMPLEX", "MPI_C_FLOAT_COMPLEX", "MPI_C_DOUBLE_COMPLEX", "MPI_DOUBLE_COMPLEX"],
    "BYTE": ["MPI_BYTE"],
    "PAIR": ["MPI_2INT", "MPI_FLOAT_INT", "MPI_DOUBLE_INT", "MPI_LONG_INT", "MPI_SHORT_INT",
             "MPI_2INTEGER", "MPI_2REAL", "MPI_2DOUBLE_PRECISION"],
}

OP_GROUPS = {
    "MPI_SUM": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "FLOATING_POINT", "COMPLEX"],
    "MPI_PROD": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "FLOATING_POINT", "COMPLEX"],
    "MPI_MAX": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "FLOATING_POINT"],
    "MPI_MIN": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "FLOATING_POINT"],
    "MPI_LAND": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "FLOATING_POINT", "LOGICAL"],
    "MPI_LOR": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "FLOATING_POINT", "LOGICAL"],
    "MPI_LXOR": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "FLOATING_POINT", "LOGICAL"],
    "MPI_BAND": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "BYTE"],
    "MPI_BOR": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "BYTE"],
    "MPI_BXOR": ["C_INTEGER", "C_INTEGER_EXTRA", "FORTRAN_INTEGER", "BYTE"],
    "MPI_MAXLOC": ["PAIR"],
    "MPI_MINLOC": ["PAIR"],
}

# types with no gfx950 representation (x87 80-bit long double)
DEVICE_UNSUPPORTED = {"MPI_LONG_DOUBLE", "MPI_C_LONG_DOUBLE_COMPLEX", "MPI_LONG_DOUBLE_INT"}


def legal_pairs():
    """Every (op, type) pair the reference accepts, excluding REPLACE/NO_OP."""
    out = []
    for op, groups in OP_GROUPS.items():
        for g in groups:
            for t in GROUPS[g]:
                out.append((op, t))
    return out
