// kernels_pair.hip — (op x kind) instantiations for kinds: K_P_2INT K_P_FLOATINT K_P_LONGINT K_P_SHORTINT K_P_DOUBLEINT K_P_2F32 K_P_2F64
#define MV2_GRP pair
#define MV2_KINDS(X) X(K_P_2INT) X(K_P_FLOATINT) X(K_P_LONGINT) X(K_P_SHORTINT) X(K_P_DOUBLEINT) X(K_P_2F32) X(K_P_2F64)
#include "group_tu.inc"
