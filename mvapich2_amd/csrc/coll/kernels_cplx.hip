// kernels_cplx.hip — (op x kind) instantiations for kinds: K_CF32_C99 K_CF64_C99 K_CF32_S K_CF64_S
#define MV2_GRP cplx
#define MV2_KINDS(X) X(K_CF32_C99) X(K_CF64_C99) X(K_CF32_S) X(K_CF64_S)
#include "group_tu.inc"
