// kernels_int32.hip — (op x kind) instantiations for kinds: K_I32 K_U32
#define MV2_GRP int32
#define MV2_KINDS(X) X(K_I32) X(K_U32)
#include "group_tu.inc"
