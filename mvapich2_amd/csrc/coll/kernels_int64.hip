// kernels_int64.hip — (op x kind) instantiations for kinds: K_I64 K_U64
#define MV2_GRP int64
#define MV2_KINDS(X) X(K_I64) X(K_U64)
#include "group_tu.inc"
