// datatype.h — builtin + derived datatype queries used by the MPI glue.
#pragma once
#include "../../../include/mpi.h"

bool dtype_valid(MPI_Datatype dt);
bool dtype_is_builtin(MPI_Datatype dt);
bool dtype_is_contiguous(MPI_Datatype dt);
// builtin types, and derived types after MPI_Type_commit (MPID_Datatype_committed_ptr)
bool dtype_committed(MPI_Datatype dt);
long dtype_true_lb(MPI_Datatype dt);
long dtype_size(MPI_Datatype dt);
long dtype_extent(MPI_Datatype dt);
// bytes from the first to one past the last byte touched by `count` elements (lb = 0)
long dtype_span(MPI_Datatype dt, int count);
// copy only the type-map bytes of `count` elements from src to dst (both laid out from
// element 0 at offset 0): what MPIR_Localcopy / Segment_unpack write into a buffer
void dtype_merge_typemap(char *dst, const char *src, MPI_Datatype dt, long count);
// MPI_Pack / MPI_Unpack of `count` elements without the position bookkeeping (no int limit
// on the packed size); either side may be device or host memory, device work is synchronous
int dtype_pack(const void *in, int count, MPI_Datatype dt, void *out);
int dtype_unpack(const void *in, int count, MPI_Datatype dt, void *out);
