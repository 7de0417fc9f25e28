// kernels_fp.hip — (op x kind) instantiations for kinds: K_F32 K_F64
#define MV2_GRP fp
#define MV2_KINDS(X) X(K_F32) X(K_F64)
#include "group_tu.inc"
