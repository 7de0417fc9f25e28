// dispatch.hip — route (op, kind) to the per-group instantiations and hold
// the op-independent data-movement pipeline (all-gather / broadcast).
#include "kernels.h"
#include "pipe.h"

#include "../common.h"

namespace mv2 {

#define MV2_GROUPS(X) X(int8) X(int16) X(int32) X(int64) X(fp) X(cplx) X(pair)

#define MV2_DECL(g)                                                                                  \
    int grp_reduce_local_##g(int, int, const void *, void *, size_t, const LaunchCfg &);             \
    int grp_reduce_n_##g(int, int, const void *const *, int, void *, size_t, const TreeParams &,     \
                         const LaunchCfg &);                                                         \
    int grp_oneshot_##g(int, int, const OneShotArgs &, const LaunchCfg &);                           \
    int grp_pipe_##g(int, int, const PipeArgs &, const LaunchCfg &);
MV2_GROUPS(MV2_DECL)
#undef MV2_DECL

// first group that recognises the kind wins (-1 = kind not in group)
#define MV2_TRY(g, fn, ...)                         \
    {                                               \
        int rc = grp_##fn##_##g(__VA_ARGS__);       \
        if (rc != -1) return rc;                    \
    }

int launch_reduce_local(int op, int kind, const void *in, void *inout, size_t count, size_t,
                        const LaunchCfg &cfg) {
#define X(g) MV2_TRY(g, reduce_local, op, kind, in, inout, count, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

int launch_reduce_n(int op, int kind, const void *const *srcs, int n, void *dst, size_t count, size_t,
                    const TreeParams &tp, const LaunchCfg &cfg) {
    if (n < 1 || n > kMaxRanks) return E_ARG;
#define X(g) MV2_TRY(g, reduce_n, op, kind, srcs, n, dst, count, tp, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

int launch_oneshot(int op, int kind, const OneShotArgs &a, size_t, const LaunchCfg &cfg) {
#define X(g) MV2_TRY(g, oneshot, op, kind, a, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

int launch_pipe_reduce(int op, int kind, const PipeArgs &a, const LaunchCfg &cfg) {
#define X(g) MV2_TRY(g, pipe, op, kind, a, cfg)
    MV2_GROUPS(X)
#undef X
    return E_TYPE;
}

int launch_pipe_copy(const PipeArgs &a, const LaunchCfg &cfg) {
    hipLaunchKernelGGL((k_pipe<NoReduce>), dim3(cfg.grid), dim3(kPipeThreads), 0, cfg.stream, a);
    return hipGetLastError() == hipSuccess ? 0 : E_INTERN;
}

}  // namespace mv2
