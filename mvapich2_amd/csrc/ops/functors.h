// functors.h — device restatement of the MPI_Op element kernels for gfx950.
//
// R<OP, KIND>::apply(a, b) returns op(a, b) with a = inoutvec (accumulator)
// and b = invec, the operand convention of MPIR_OP_TYPE_REDUCE_CASE
// (reference src/include/oputil.h:50-57).  Results are bit-identical to the
// reference's host loops compiled by gcc -O2 on x86-64:
//   * integer SUM/PROD wrap modulo 2^bits (the gcc loop's behaviour, Appendix A.10)
//   * MAX/MIN use MPIR_MAX/MPIR_MIN NaN-skipping, tie-keeps-a (mpiimpl.h:4034-4040)
//   * logical ops store 0/1 in the element type, floats included (opland.c:73-76)
//   * struct complex PROD follows opprod.c:43-54; C99 _Complex PROD follows
//     C99 Annex G (the libgcc __mulsc3/__muldc3 algorithm gcc calls)
//   * MAXLOC/MINLOC follow MPIR_MAXLOC_C_CASE / MPIR_MINLOC_C_CASE
//     (opmaxloc.c:65-87, opminloc.c:65-87) and the Fortran pair case (:89-111)
// Kernels are compiled with -ffp-contract=off so no a*b+c is fused (x86-64
// gcc -O2 does not contract either).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "../common.h"

namespace mv2 {

struct cf32 { float re, im; };
struct cf64 { double re, im; };
struct p2int { int value; int loc; };
struct pfloatint { float value; int loc; };
struct plongint { long value; int loc; };     // sizeof 16 (12 data + 4 pad)
struct pshortint { short value; int loc; };   // sizeof 8 (value@0, loc@4)
struct pdoubleint { double value; int loc; }; // sizeof 16 (12 data + 4 pad)
struct p2f32 { float value; float loc; };
struct p2f64 { double value; double loc; };

static_assert(sizeof(plongint) == 16 && sizeof(pdoubleint) == 16 && sizeof(pshortint) == 8, "pair layout");

template <int K> struct KT;
template <> struct KT<K_I8> { using T = int8_t; };
template <> struct KT<K_U8> { using T = uint8_t; };
template <> struct KT<K_I16> { using T = int16_t; };
template <> struct KT<K_U16> { using T = uint16_t; };
template <> struct KT<K_I32> { using T = int32_t; };
template <> struct KT<K_U32> { using T = uint32_t; };
template <> struct KT<K_I64> { using T = int64_t; };
template <> struct KT<K_U64> { using T = uint64_t; };
template <> struct KT<K_F32> { using T = float; };
template <> struct KT<K_F64> { using T = double; };
template <> struct KT<K_CF32_C99> { using T = cf32; };
template <> struct KT<K_CF64_C99> { using T = cf64; };
template <> struct KT<K_CF32_S> { using T = cf32; };
template <> struct KT<K_CF64_S> { using T = cf64; };
template <> struct KT<K_P_2INT> { using T = p2int; };
template <> struct KT<K_P_FLOATINT> { using T = pfloatint; };
template <> struct KT<K_P_LONGINT> { using T = plongint; };
template <> struct KT<K_P_SHORTINT> { using T = pshortint; };
template <> struct KT<K_P_DOUBLEINT> { using T = pdoubleint; };
template <> struct KT<K_P_2F32> { using T = p2f32; };
template <> struct KT<K_P_2F64> { using T = p2f64; };

// MPIR_MAX / MPIR_MIN (mpiimpl.h:4034-4040)
template <typename T> __device__ __forceinline__ T mpir_max(T a, T b) {
    return (a != a && b != b) ? a : ((a != a && b == b) ? b : ((a == a && b != b) ? a : ((b > a) ? b : a)));
}
template <typename T> __device__ __forceinline__ T mpir_min(T a, T b) {
    return (a != a && b != b) ? a : ((a != a && b == b) ? b : ((a == a && b != b) ? a : ((a > b) ? b : a)));
}

// modular integer arithmetic (no signed-overflow UB on the device either)
template <typename T> __device__ __forceinline__ T wadd(T a, T b) {
    using U = typename std::make_unsigned<T>::type;
    using W = typename std::conditional<(sizeof(T) <= 4), uint32_t, uint64_t>::type;
    return (T)(U)((W)(U)a + (W)(U)b);
}
template <typename T> __device__ __forceinline__ T wmul(T a, T b) {
    using U = typename std::make_unsigned<T>::type;
    using W = typename std::conditional<(sizeof(T) <= 4), uint32_t, uint64_t>::type;
    return (T)(U)((W)(U)a * (W)(U)b);
}

// ---- x86-64 SSE NaN semantics for the reference's fp arithmetic ----
// A NaN result of `a op b` on x86 SSE (the reference's host loops, gcc -O2)
// is the first operand's NaN quieted if a is NaN, else b's NaN quieted,
// else the x86 default NaN (sign bit set).  gfx950 returns its own
// canonical NaN, so the result is rewritten bit-exactly.
template <typename F> struct FBits;
template <> struct FBits<float> { using U = uint32_t; static constexpr U quiet = 0x00400000u, dflt = 0xFFC00000u; };
template <> struct FBits<double> { using U = uint64_t; static constexpr U quiet = 0x0008000000000000ull, dflt = 0xFFF8000000000000ull; };

template <typename F> __device__ __forceinline__ F x86_nan(F r, F a, F b) {
    using B = FBits<F>;
    if (!__builtin_isnan(r)) return r;
    typename B::U u;
    if (__builtin_isnan(a)) u = __builtin_bit_cast(typename B::U, a) | B::quiet;
    else if (__builtin_isnan(b)) u = __builtin_bit_cast(typename B::U, b) | B::quiet;
    else u = B::dflt;
    return __builtin_bit_cast(F, u);
}
template <typename F> __device__ __forceinline__ F fadd(F a, F b) { return x86_nan<F>(a + b, a, b); }
template <typename F> __device__ __forceinline__ F fsub(F a, F b) { return x86_nan<F>(a - b, a, b); }
template <typename F> __device__ __forceinline__ F fmul(F a, F b) { return x86_nan<F>(a * b, a, b); }

// C99 Annex G complex multiply (the libgcc __mulsc3 / __muldc3 algorithm)
template <typename F> __device__ __forceinline__ void annexg_mul(F a, F b, F c, F d, F &x, F &y) {
    F ac = fmul(a, c), bd = fmul(b, d), ad = fmul(a, d), bc = fmul(b, c);
    x = fsub(ac, bd);
    y = fadd(ad, bc);
    if (__builtin_isnan(x) && __builtin_isnan(y)) {
        bool recalc = false;
        if (__builtin_isinf(a) || __builtin_isinf(b)) {
            a = __builtin_copysign(__builtin_isinf(a) ? (F)1 : (F)0, a);
            b = __builtin_copysign(__builtin_isinf(b) ? (F)1 : (F)0, b);
            if (__builtin_isnan(c)) c = __builtin_copysign((F)0, c);
            if (__builtin_isnan(d)) d = __builtin_copysign((F)0, d);
            recalc = true;
        }
        if (__builtin_isinf(c) || __builtin_isinf(d)) {
            c = __builtin_copysign(__builtin_isinf(c) ? (F)1 : (F)0, c);
            d = __builtin_copysign(__builtin_isinf(d) ? (F)1 : (F)0, d);
            if (__builtin_isnan(a)) a = __builtin_copysign((F)0, a);
            if (__builtin_isnan(b)) b = __builtin_copysign((F)0, b);
            recalc = true;
        }
        if (!recalc && (__builtin_isinf(ac) || __builtin_isinf(bd) || __builtin_isinf(ad) || __builtin_isinf(bc))) {
            if (__builtin_isnan(a)) a = __builtin_copysign((F)0, a);
            if (__builtin_isnan(b)) b = __builtin_copysign((F)0, b);
            if (__builtin_isnan(c)) c = __builtin_copysign((F)0, c);
            if (__builtin_isnan(d)) d = __builtin_copysign((F)0, d);
            recalc = true;
        }
        if (recalc) {
            const F inf = (F)__builtin_inf();
            x = fmul(inf, fsub(fmul(a, c), fmul(b, d)));
            y = fmul(inf, fadd(fmul(a, d), fmul(b, c)));
        }
    }
}

template <int OP, int K, typename Enable = void> struct R;

// ---------------- scalar integer / floating kinds ----------------
template <int K> constexpr bool is_int_kind() { return K >= K_I8 && K <= K_U64; }
template <int K> constexpr bool is_fp_kind() { return K == K_F32 || K == K_F64; }
template <int K> constexpr bool is_scalar_kind() { return is_int_kind<K>() || is_fp_kind<K>(); }

// kOrderFree: the reduction order cannot change a single result bit, so the kernels evaluate any
// algorithm's order as the LINEAR chain and the order-specialised bodies are not instantiated
// (code size: libmpi.so's gfx950 code objects).  True for the integer kinds -- wrapping SUM / PROD,
// MAX / MIN, the logical and the bitwise ops are all exactly associative and commutative -- and
// for MPI_2INT MAXLOC / MINLOC (the largest / smallest value with the smallest loc among its ties,
// and no padding bytes whose source would depend on the order).  Floating point, complex and the
// padded pair kinds keep every order.
template <int OP, int K>
struct R<OP, K, typename std::enable_if<is_scalar_kind<K>()>::type> {
    using T = typename KT<K>::T;
    static constexpr bool kOrderFree = is_int_kind<K>();
    static __device__ __forceinline__ T apply(T a, T b) {
        if constexpr (OP == OP_SUM) {
            if constexpr (is_int_kind<K>()) return wadd(a, b); else return fadd(a, b);
        } else if constexpr (OP == OP_PROD) {
            if constexpr (is_int_kind<K>()) return wmul(a, b); else return fmul(a, b);
        } else if constexpr (OP == OP_MAX) {
            return mpir_max(a, b);
        } else if constexpr (OP == OP_MIN) {
            return mpir_min(a, b);
        } else if constexpr (OP == OP_LAND) {
            return (T)((a != (T)0) && (b != (T)0));
        } else if constexpr (OP == OP_LOR) {
            return (T)((a != (T)0) || (b != (T)0));
        } else if constexpr (OP == OP_LXOR) {
            return (T)(((a != (T)0) && !(b != (T)0)) || (!(a != (T)0) && (b != (T)0)));
        } else if constexpr (OP == OP_BAND) {
            return (T)(a & b);
        } else if constexpr (OP == OP_BOR) {
            return (T)(a | b);
        } else if constexpr (OP == OP_BXOR) {
            return (T)(a ^ b);
        } else {
            static_assert(OP < 0, "invalid op for scalar kind");
        }
    }
};

// ---------------- complex kinds ----------------
template <int OP, int K>
struct R<OP, K, typename std::enable_if<(K >= K_CF32_C99 && K <= K_CF64_S)>::type> {
    using T = typename KT<K>::T;
    static constexpr bool kOrderFree = false;
    static __device__ __forceinline__ T apply(T a, T b) {
        T r;
        if constexpr (OP == OP_SUM) {
            r.re = fadd(a.re, b.re);
            r.im = fadd(a.im, b.im);
        } else if constexpr (OP == OP_PROD) {
            if constexpr (K == K_CF32_S || K == K_CF64_S) {
                // opprod.c:50-51: c = a; re = c.re*b.re - c.im*b.im; im = c.im*b.re + c.re*b.im
                r.re = fsub(fmul(a.re, b.re), fmul(a.im, b.im));
                r.im = fadd(fmul(a.im, b.re), fmul(a.re, b.im));
            } else {
                annexg_mul(a.re, a.im, b.re, b.im, r.re, r.im);
            }
        } else {
            static_assert(OP < 0, "invalid op for complex kind");
        }
        return r;
    }
};

// ---------------- MAXLOC / MINLOC pair kinds ----------------
template <int OP, int K>
struct R<OP, K, typename std::enable_if<(K >= K_P_2INT && K <= K_P_2F64)>::type> {
    using T = typename KT<K>::T;
    static constexpr bool kOrderFree = K == K_P_2INT;
    static __device__ __forceinline__ T apply(T a, T b) {
        static_assert(OP == OP_MAXLOC || OP == OP_MINLOC, "pair kinds take MAXLOC/MINLOC");
        const bool an = a.value != a.value, bn = b.value != b.value;
        if (an && bn) {
            a.loc = mpir_min(a.loc, b.loc);
        } else if (an && !bn) {
            a.value = b.value;
            a.loc = b.loc;
        } else if (!an && bn) {
        } else {
            if constexpr (OP == OP_MAXLOC) {
                if (a.value < b.value) { a.value = b.value; a.loc = b.loc; }
                else if (a.value <= b.value) a.loc = mpir_min(a.loc, b.loc);
            } else {
                if (a.value > b.value) { a.value = b.value; a.loc = b.loc; }
                else if (a.value >= b.value) a.loc = mpir_min(a.loc, b.loc);
            }
        }
        return a;
    }
};

// compile-time legality of (OP, KIND): mirrors op_valid_for_groups on kinds
template <int OP, int K> constexpr bool legal() {
    if (OP == OP_MAXLOC || OP == OP_MINLOC) return K >= K_P_2INT && K <= K_P_2F64;
    if (K >= K_P_2INT) return false;
    if (K >= K_CF32_C99 && K <= K_CF64_S) return OP == OP_SUM || OP == OP_PROD;
    if (is_fp_kind<K>()) return OP != OP_BAND && OP != OP_BOR && OP != OP_BXOR && OP < OP_MINLOC;
    if (is_int_kind<K>()) return OP < OP_MINLOC;
    return false;
}

// The kind an (OP, K) pair is instantiated with.  Signed and unsigned integers of one width give
// the same bits under every op but MAX / MIN (two's-complement wrapping SUM / PROD, the logical
// ops' 0 / 1, the bitwise ops), and the struct and C99 complex kinds the same SUM, so those pairs
// share one instantiation: the signed kind runs as its unsigned twin, struct complex SUM as C99.
template <int OP, int K> constexpr int canon_kind() {
    if constexpr (is_int_kind<K>()) {
        if (OP != OP_MAX && OP != OP_MIN && (K == K_I8 || K == K_I16 || K == K_I32 || K == K_I64)) return K + 1;
        return K;
    } else if constexpr (K == K_CF32_S || K == K_CF64_S) {
        return OP == OP_SUM ? K - 2 : K;
    } else {
        return K;
    }
}
static_assert(K_U8 == K_I8 + 1 && K_U64 == K_I64 + 1 && K_CF32_C99 == K_CF32_S - 2 && K_CF64_C99 == K_CF64_S - 2,
              "canon_kind relies on the Kind order");

}  // namespace mv2
