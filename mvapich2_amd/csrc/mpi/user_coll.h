// user_coll.h — reductions the library evaluates on the host: user MPI_Op
// functions (MPI_Op_create) and builtin ops on x87 80-bit types, which gfx950
// cannot represent.  Each follows the algorithm the reference selects for the
// call (orders.cpp plans) with the function applied as uop(in, inout), like the
// reference's own host loops (allreduce_osu.c:3925-3958 ring, :360-630 RD, ...).
#pragma once
#include <stddef.h>

#include "../../../include/mpi.h"

namespace mv2 {

// Pinned host staging kept per slot and grown on demand (no page faults or zero fill per
// call; device copies run as DMA).  Used under the global critical section.
enum HostSlot { HS_IN, HS_INOUT, HS_PACKED, HS_OPERANDS, HS_RESULT, HS_PARTIALS, HS_COUNT };
class HostBuf {
  public:
    explicit HostBuf(int slot) : slot_(slot) {}
    void resize(size_t n);
    char *data() { return p_; }
    const char *data() const { return p_; }
    size_t size() const { return n_; }

  private:
    int slot_;
    char *p_ = nullptr;
    size_t n_ = 0;
};

struct HostOp {
    MPI_User_function *fn;
    int opk;  // OpKind (orders.h): builtin (x87), commutative or non-commutative user op
};

// MPI_Allreduce / MPI_Reduce / MPI_Reduce_scatter on one node; buffers may be device or host
// memory; count / counts > 0.  Return an MPI error class.
int host_allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, const HostOp &op);
int host_reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, const HostOp &op, int root);
int host_reduce_scatter(const void *sendbuf, void *recvbuf, const int *counts, MPI_Datatype dt, const HostOp &op);

}  // namespace mv2
