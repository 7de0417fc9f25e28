// kernels_int8.hip — (op x kind) instantiations for kinds: K_I8 K_U8
#define MV2_GRP int8
#define MV2_KINDS(X) X(K_I8) X(K_U8)
#include "group_tu.inc"
