// kernels_int16.hip — (op x kind) instantiations for kinds: K_I16 K_U16
#define MV2_GRP int16
#define MV2_KINDS(X) X(K_I16) X(K_U16)
#include "group_tu.inc"
