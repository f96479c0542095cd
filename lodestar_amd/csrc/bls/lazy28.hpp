// Lazily reduced Fp in 14 signed digits of 28 bits, Montgomery form with R' = 2^392, for
// the long product chains (exponentiations, Miller loops).
//
// Why: the 28-bit-digit Montgomery product is the device's Fp product (field.hpp
// fp_mul_d28_lazy), but on 12 x 32-bit limbs each call re-cuts both operands into
// digits, packs its result back into limbs and subtracts p once more -- ~95 of its ~580
// VALU instructions -- and every addition and subtraction around it carries through 12
// limbs and reduces (~36 instructions).  Here an element STAYS in digit form:
//   * value = sum d_k 2^(28 k) with signed 32-bit digits, any representative of its class
//     whose magnitude is below a tracked multiple of p (negative values included);
//   * a + b and a - b are 14 adds / subtracts, digit by digit, no carries, no reduction;
//   * the product takes the digits as they are (signed 32 x 32 -> 64-bit multiply-adds)
//     and returns normalised digits (0..12 in [0, 2^28), the top one signed): with
//     R' = 2^392 = 2^(28 * 14) the 14 reduction steps leave the result digit-aligned, so
//     no re-cut or pack, and since 2^392 / p > 2520 its magnitude is < p (1 + Va Vb /
//     2520): no final subtraction.
// The bounds are part of the type: Lz<D, V> has |digit| <= D and |value| < V p.  Every
// operation computes its result's bounds at compile time and static_asserts its
// preconditions (the product's signed 64-bit columns cannot overflow, digits fit 31 bits
// and a sign), so a formula that could overflow does not compile; lz_norm() propagates
// the carries where a formula needs smaller digits.
//
// Conversions at kernel boundaries: from a canonical 12 x 32-bit Montgomery Fp (R = 2^384)
// by re-cutting its bits 8 to the left (the integer A 2^8 is a representative of a R',
// value < 256 p, no product); back by one product with the constant 2^384 (x 2^384 / R'
// = a R), a sign fix, a pack and one conditional subtraction.
//
// Test: tests/test_lazy28.py (the raw product at its digit bounds against big integers,
// every operation and the tower functions against field arithmetic, bit-exact after the
// conversion back).
#pragma once

#include "field.hpp"  // (field.hpp includes this header after its Fp basics)

#if defined(BLS_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
extern unsigned long long bls_lz_norm_counter;  // host-only: carry passes (tests, work model)
#define LZ_COUNT_NORM() (++bls_lz_norm_counter)
#else
#define LZ_COUNT_NORM() ((void)0)
#endif

namespace bls {

#define LZ_M28 0xFFFFFFFll

// ---- compile-time tables ---------------------------------------------------------
constexpr int64_t lz_p28(int k) {
  const int64_t t[14] = {0xfffaaab, 0xfefffff, 0x3ffffb9, 0xfffeb15, 0x6241eab, 0xa0f6b0f, 0xf6730d2,
                         0xf38512b, 0x4774b84, 0x4bacd76, 0xba7b643, 0xe69a4b1, 0x1ea397f, 0x001a011};
  return t[k];
}
constexpr int64_t lz_max(int64_t a, int64_t b) { return a > b ? a : b; }
// |value| < V p  ->  |top digit| <= V (p >> 364) + V (digits 0..12 normalised)
constexpr int64_t lz_top_norm(int64_t v) { return v * 106514ll; }
// 2^392 / p = 2520.2: a product of |values| < Va p and < Vb p is < (1 + ceil(Va Vb / 2520)) p
constexpr int64_t lz_mul_v(int64_t va, int64_t vb) { return 1 + (va * vb + 2519) / 2520; }
// the product's largest column: 14 digit products of the operands, 14 of m_i p_j (< 2^56
// each), the carry from below (< 2^36); signed 64-bit
constexpr bool lz_mul_fits(int64_t da, int64_t db) {
  return (double)da * (double)db * 14.0 + 14.0 * (double)LZ_M28 * (double)LZ_M28 + 68719476736.0 <
         9223372036854775807.0 * 0.999;
}

template <int64_t D, int64_t V>
struct Lz {
  static constexpr int64_t DM = D;  // |every digit| <= DM
  static constexpr int64_t VM = V;  // |value| < VM p
  static_assert(D >= 0 && D <= 0x7FFFFFFFll, "digits are signed 32-bit");
  static_assert(V >= 1 && V <= 2520, "value bound");
  int32_t d[14];
};

template <class To, class From>
BLS_HD To lz_widen(const From& x) {
  static_assert(From::DM <= To::DM && From::VM <= To::VM, "lz_widen narrows");
  To r;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.d[k] = x.d[k];
  return r;
}
template <class A, class B>
using LzMax = Lz<lz_max(A::DM, B::DM), lz_max(A::VM, B::VM)>;

// ---- additive operations (inline: 14 VALU instructions, no reduction) -----------------
// lz_norm (below) first brings an operand's digits back to 28 bits when the sum's digits
// would not fit 31 bits (with room for a later carry pass)
#define LZ_DMAX (0x7FFFFFFFll - 16)
template <int64_t D, int64_t V>
BLS_HD Lz<lz_max(LZ_M28, lz_top_norm(V)), V> lz_norm(const Lz<D, V>& a);
template <int64_t D1, int64_t V1, int64_t D2, int64_t V2>
BLS_HD auto lz_add(const Lz<D1, V1>& a, const Lz<D2, V2>& b) {
  if constexpr (D1 + D2 <= LZ_DMAX) {
    Lz<D1 + D2, V1 + V2> r;
#pragma unroll
    for (int k = 0; k < 14; ++k) r.d[k] = a.d[k] + b.d[k];
    return r;
  } else if constexpr (D1 >= D2) {
    return lz_add(lz_norm(a), b);
  } else {
    return lz_add(a, lz_norm(b));
  }
}
template <int64_t D1, int64_t V1, int64_t D2, int64_t V2>
BLS_HD auto lz_sub(const Lz<D1, V1>& a, const Lz<D2, V2>& b) {
  if constexpr (D1 + D2 <= LZ_DMAX) {
    Lz<D1 + D2, V1 + V2> r;
#pragma unroll
    for (int k = 0; k < 14; ++k) r.d[k] = a.d[k] - b.d[k];
    return r;
  } else if constexpr (D1 >= D2) {
    return lz_sub(lz_norm(a), b);
  } else {
    return lz_sub(a, lz_norm(b));
  }
}
template <int64_t D, int64_t V>
BLS_HD Lz<D, V> lz_neg(const Lz<D, V>& a) {
  Lz<D, V> r;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.d[k] = -a.d[k];
  return r;
}
template <int64_t D, int64_t V>
BLS_HD auto lz_dbl(const Lz<D, V>& a) {
  return lz_add(a, a);
}
// small constant multiple (digit-wise)
template <int64_t C, int64_t D, int64_t V>
BLS_HD auto lz_mulc(const Lz<D, V>& a) {
  if constexpr (C * D <= LZ_DMAX) {
    Lz<C * D, C * V> r;
#pragma unroll
    for (int k = 0; k < 14; ++k) r.d[k] = (int32_t)C * a.d[k];
    return r;
  } else {
    static_assert(D > LZ_M28, "C (2^28 - 1) must fit 31 bits");
    return lz_mulc<C>(lz_norm(a));
  }
}

// carries propagated: digits 0..12 in [0, 2^28), the top digit signed, the value unchanged
template <int64_t V>
using LzN = Lz<lz_max(LZ_M28, lz_top_norm(V)), V>;
template <int64_t D, int64_t V>
BLS_HD Lz<lz_max(LZ_M28, lz_top_norm(V)), V> lz_norm(const Lz<D, V>& a) {
  static_assert(D <= LZ_DMAX, "carry room");
  LZ_COUNT_NORM();
  LzN<V> r;
  int32_t c = 0;
#pragma unroll
  for (int k = 0; k < 13; ++k) {
    const int32_t t = a.d[k] + c;
    r.d[k] = t & (int32_t)LZ_M28;
    c = t >> 28;  // arithmetic
  }
  r.d[13] = a.d[13] + c;
  return r;
}
// a product's output: normalised digits, |value| < 2 p
typedef LzN<2> LzP;

// Value reduction in one carry pass: q ~ value / p from the top digit alone (value =
// d13 2^364 + L with |L| < 2^31 2^337, i.e. < 2^-13 p), then the digits of value - q p
// with carries (64-bit per digit: |q p_k| < 2^40).  q = floor(d13 C / 2^32) with C =
// floor(2^396 / p) = 40323 is at most ~1.03 below value / p and never above it by more
// than 0.03: the result is in (-p/32, 1.1 p).
// ~5 VALU instructions a digit; what keeps a loop-carried value (the Miller loop's f)
// from growing past the bounds its next products need.
#define LZ_QC 40323ll
template <int64_t D, int64_t V>
BLS_HD LzN<2> lz_reduce(const Lz<D, V>& a) {
  const int32_t q = (int32_t)(((int64_t)a.d[13] * LZ_QC) >> 32);
  LzN<2> r;
  int32_t c = 0;
#pragma unroll
  for (int k = 0; k < 13; ++k) {
    const int64_t t = (int64_t)a.d[k] + c - (int64_t)q * lz_p28(k);
    r.d[k] = (int32_t)((uint32_t)t & (uint32_t)LZ_M28);
    c = (int32_t)(t >> 28);
  }
  r.d[13] = (int32_t)((int64_t)a.d[13] + c - (int64_t)q * lz_p28(13));
  return r;
}

// a / 2 mod p: (a + (a odd ? p : 0)) / 2, halved digit by digit (each digit's low bit
// moves down as 2^27 into the digit below; the value's parity is digit 0's)
template <int64_t D, int64_t V>
BLS_HD auto lz_half(const Lz<D, V>& a) {
  if constexpr (D + LZ_M28 <= LZ_DMAX) {
    const int32_t mask = -(a.d[0] & 1);
    int32_t s[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) s[k] = a.d[k] + ((int32_t)lz_p28(k) & mask);
    Lz<(D + LZ_M28) / 2 + (1ll << 27), V> r;
#pragma unroll
    for (int k = 0; k < 13; ++k) r.d[k] = (s[k] >> 1) + ((s[k + 1] & 1) << 27);
    r.d[13] = s[13] >> 1;
    return r;
  } else {
    return lz_half(lz_norm(a));
  }
}

// ---- the product -----------------------------------------------------------------
// t = x y over 14 x 14 signed digits (27 columns of signed 64 bits), then 14 Montgomery
// steps of 28 bits: m_i = t_i (-1/p) mod 2^28 (the column's low bits, two's complement),
// t += m_i p 2^(28 i), t_i's carry (arithmetic shift) into t_{i+1}; the result is columns
// 14..27 normalised.  392 multiply-adds, ~490 VALU instructions.
#define LZ_NP28 0xFFCFFFDu  // -p^-1 mod 2^28
BLS_HD void lz_redc(int64_t t[28], int32_t r[14]) {
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t m = ((uint32_t)t[i] * LZ_NP28) & (uint32_t)LZ_M28;
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] = (int64_t)((uint64_t)t[i + j] + (uint64_t)m * (uint32_t)lz_p28(j));
    t[i + 1] += t[i] >> 28;
  }
#pragma unroll
  for (int k = 14; k < 27; ++k) {
    r[k - 14] = (int32_t)((uint32_t)t[k] & (uint32_t)LZ_M28);
    t[k + 1] += t[k] >> 28;
  }
  r[13] = (int32_t)t[27];
}

BLS_HD void lz_mul_core(const int32_t x[14], const int32_t y[14], int32_t r[14]) {
  BLS_COUNT_FPM();
  int64_t t[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] += (int64_t)x[i] * y[j];
  lz_redc(t, r);
}

// squaring: 14 squares + 91 cross products against doubled digits
BLS_HD void lz_sqr_core(const int32_t x[14], int32_t r[14]) {
  BLS_COUNT_FPM();
  int32_t x2[14];
#pragma unroll
  for (int k = 0; k < 14; ++k) x2[k] = x[k] * 2;
  int64_t t[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    t[2 * i] += (int64_t)x[i] * x[i];
#pragma unroll
    for (int j = i + 1; j < 14; ++j) t[i + j] += (int64_t)x2[i] * x[j];
  }
  lz_redc(t, r);
}

struct Lz14 {
  int32_t d[14];
};
// Out of line on the device, operands as 28 scalar words (the calling convention hands
// them over in v0-v27 and returns the 14 digits in v0-v13; a struct argument would go
// through private memory, field.hpp fp_mul_w)
#define LZ_W14(x) int32_t x##0, int32_t x##1, int32_t x##2, int32_t x##3, int32_t x##4, int32_t x##5, \
                  int32_t x##6, int32_t x##7, int32_t x##8, int32_t x##9, int32_t x##10, int32_t x##11, \
                  int32_t x##12, int32_t x##13
#define LZ_ARR(x) {x##0, x##1, x##2, x##3, x##4, x##5, x##6, x##7, x##8, x##9, x##10, x##11, x##12, x##13}
#define LZ_L14(v) (v).d[0], (v).d[1], (v).d[2], (v).d[3], (v).d[4], (v).d[5], (v).d[6], (v).d[7], (v).d[8], \
                  (v).d[9], (v).d[10], (v).d[11], (v).d[12], (v).d[13]
BLS_NOINLINE Lz14 lz_mul_w(LZ_W14(a), LZ_W14(b)) {
  const int32_t x[14] = LZ_ARR(a), y[14] = LZ_ARR(b);
  Lz14 r;
  lz_mul_core(x, y, r.d);
  return r;
}
BLS_NOINLINE Lz14 lz_sqr_w(LZ_W14(a)) {
  const int32_t x[14] = LZ_ARR(a);
  Lz14 r;
  lz_sqr_core(x, r.d);
  return r;
}

// the product; an operand whose digits would overflow the columns is normalised first
// (the larger one, then the other if still needed: 40 VALU each, decided at compile time)
template <int64_t D1, int64_t V1, int64_t D2, int64_t V2>
BLS_HD LzN<lz_mul_v(V1, V2)> lz_mul(const Lz<D1, V1>& a, const Lz<D2, V2>& b) {
  if constexpr (lz_mul_fits(D1, D2)) {
    const Lz14 t = lz_mul_w(LZ_L14(a), LZ_L14(b));
    LzN<lz_mul_v(V1, V2)> r;
#pragma unroll
    for (int k = 0; k < 14; ++k) r.d[k] = t.d[k];
    return r;
  } else if constexpr (D1 >= D2 && D1 > LZ_M28) {
    return lz_mul(lz_norm(a), b);
  } else {
    static_assert(D2 > LZ_M28, "normalised operands always fit");
    return lz_mul(a, lz_norm(b));
  }
}
template <int64_t D, int64_t V>
BLS_HD LzN<lz_mul_v(V, V)> lz_sqr(const Lz<D, V>& a) {
  if constexpr (2 * D <= 0x7FFFFFFFll && lz_mul_fits(D, D)) {
    const Lz14 t = lz_sqr_w(LZ_L14(a));
    LzN<lz_mul_v(V, V)> r;
#pragma unroll
    for (int k = 0; k < 14; ++k) r.d[k] = t.d[k];
    return r;
  } else {
    return lz_sqr(lz_norm(a));
  }
}

// ---- conversions ---------------------------------------------------------------------
typedef LzN<256> LzIn;

// canonical 12-limb Montgomery Fp (a 2^384 mod p, < p) -> digits of a 2^384 2^8 (a
// representative of a R', < 256 p): bits 28 k - 8 .. 28 k + 19 of the limbs
BLS_HD LzIn lz_from_fp(const Fp& a) {
  LzIn r;
  r.d[0] = (int32_t)((a.l[0] << 8) & (uint32_t)LZ_M28);
#pragma unroll
  for (int k = 1; k < 14; ++k) {
    const int o = 28 * k - 8, w = o >> 5, s = o & 31;
    const uint64_t pair = ((uint64_t)(w + 1 < 12 ? a.l[w + 1] : 0u) << 32) | a.l[w];
    r.d[k] = (int32_t)((uint32_t)(pair >> s) & (uint32_t)LZ_M28);
  }
  return r;
}

// 2^384 mod p as digits (the constant that takes x R' back to x R)
BLS_HD Lz<LZ_M28, 1> lz_c384() {
  const int32_t t[14] = {0x2fffd, 0x900000, 0xc000276, 0xbc40, 0x8baebf4, 0x5753c75, 0x55f4898,
                         0x7052574, 0x7ce5853, 0x56ec6d7, 0x71a97a2, 0xe4935c0, 0xec3fa80, 0x15f65};
  Lz<LZ_M28, 1> r;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.d[k] = t[k];
  return r;
}

// R' mod p (the lazy form of 1); lz_mul(x, lz_one()) brings any x to |value| < 2 p
BLS_HD Lz<LZ_M28, 1> lz_one() {
  const int32_t t[14] = {0x347fcb8, 0xd800000, 0x2b119, 0xcde6d2, 0xc7212e0, 0x83a2090, 0x37669f,
                         0xda0f73e, 0x9b09b42, 0x1297bb0, 0x515d98f, 0x12ca7c, 0x659fcfa, 0x577a};
  Lz<LZ_M28, 1> r;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.d[k] = t[k];
  return r;
}
BLS_HD Lz<LZ_M28, 1> lz_zero() {
  Lz<LZ_M28, 1> r;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.d[k] = 0;
  return r;
}

// any lazy value -> canonical 12-limb Montgomery Fp (R = 2^384)
template <int64_t D, int64_t V>
BLS_HD Fp lz_to_fp(const Lz<D, V>& x) {
  const auto y = lz_mul(x, lz_c384());  // x 2^384 / 2^392 = a 2^384 mod p, in (-p, 2p)
  static_assert(decltype(y)::VM <= 2, "one correction of p");
  // negative (top digit < 0): + p; then carries, 12 limbs, one conditional subtraction
  const int32_t neg = y.d[13] >> 31;
  int32_t c = 0;
  uint32_t z[14];
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int32_t t = y.d[k] + ((int32_t)lz_p28(k) & neg) + c;
    z[k] = (uint32_t)t & (uint32_t)LZ_M28;
    c = t >> 28;
  }
  Fp r;
  uint64_t acc = 0;
  int nb = 0, w = 0;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    acc |= (uint64_t)z[k] << nb;
    nb += 28;
    while (nb >= 32 && w < 12) {
      r.l[w++] = (uint32_t)acc;
      acc >>= 32;
      nb -= 32;
    }
  }
  while (w < 12) {
    r.l[w++] = (uint32_t)acc;
    acc >>= 32;
  }
  return fp_reduce_once(r);
}

// a^e for a fixed exponent (limb accessor E, wave-uniform, MSB first): field.hpp
// fp_pow_const's sliding window of width 4 over the odd powers a, a^3, .., a^15, every
// product in the lazy form; one conversion in, one product out.  The operands' types
// close at V = 256: a product of two values < 256 p is < 28 p.
template <uint32_t (*E)(int), int BITS>
BLS_HD Fp lz_pow_const(const Fp& a_in) {
  typedef LzIn T;
  T tab[8];
  tab[0] = lz_from_fp(a_in);
  const T a2 = lz_widen<T>(lz_sqr(tab[0]));
  for (int k = 1; k < 8; ++k) tab[k] = lz_widen<T>(lz_mul(tab[k - 1], a2));
  T r = tab[0];
  bool started = false;
  int i = BITS - 1;
  while (i >= 0) {
    if (!((E(i >> 5) >> (i & 31)) & 1u)) {
      r = lz_widen<T>(lz_sqr(r));
      --i;
      continue;
    }
    int j = i - 3 < 0 ? 0 : i - 3;
    while (!((E(j >> 5) >> (j & 31)) & 1u)) ++j;
    uint32_t val = 0;
    for (int k = i; k >= j; --k) {
      val = (val << 1) | ((E(k >> 5) >> (k & 31)) & 1u);
      if (started) r = lz_widen<T>(lz_sqr(r));
    }
    r = started ? lz_widen<T>(lz_mul(r, tab[val >> 1])) : tab[val >> 1];
    started = true;
    i = j - 1;
  }
  return lz_to_fp(r);
}

// ---- Fp2 over lazy coefficients -----------------------------------------------------
template <class T>
struct L2 {
  T c0, c1;
};
template <class A, class B>
BLS_HD L2<LzMax<A, B>> l2_join(const A& c0, const B& c1) {
  typedef LzMax<A, B> T;
  return L2<T>{lz_widen<T>(c0), lz_widen<T>(c1)};
}
template <class To, class A>
BLS_HD L2<To> l2_widen(const L2<A>& a) {
  return L2<To>{lz_widen<To>(a.c0), lz_widen<To>(a.c1)};
}
template <class A, class B>
BLS_HD auto l2_add(const L2<A>& a, const L2<B>& b) {
  return l2_join(lz_add(a.c0, b.c0), lz_add(a.c1, b.c1));
}
template <class A, class B>
BLS_HD auto l2_sub(const L2<A>& a, const L2<B>& b) {
  return l2_join(lz_sub(a.c0, b.c0), lz_sub(a.c1, b.c1));
}
template <class A>
BLS_HD L2<A> l2_neg(const L2<A>& a) {
  return L2<A>{lz_neg(a.c0), lz_neg(a.c1)};
}
template <class A>
BLS_HD auto l2_dbl(const L2<A>& a) {
  return l2_add(a, a);
}
template <int64_t C, class A>
BLS_HD auto l2_mulc(const L2<A>& a) {
  return l2_join(lz_mulc<C>(a.c0), lz_mulc<C>(a.c1));
}
template <class A>
BLS_HD auto l2_norm(const L2<A>& a) {
  return l2_join(lz_norm(a.c0), lz_norm(a.c1));
}
template <class A>
BLS_HD L2<LzN<2>> l2_reduce(const L2<A>& a) {
  return L2<LzN<2>>{lz_reduce(a.c0), lz_reduce(a.c1)};
}
template <class A>
BLS_HD auto l2_half(const L2<A>& a) {
  return l2_join(lz_half(a.c0), lz_half(a.c1));
}
template <class A>
BLS_HD L2<A> l2_conj(const L2<A>& a) {
  return L2<A>{a.c0, lz_neg(a.c1)};
}
// a (1 + u) = (a0 - a1, a0 + a1)
template <class A>
BLS_HD auto l2_mul_xi(const L2<A>& a) {
  return l2_join(lz_sub(a.c0, a.c1), lz_add(a.c0, a.c1));
}
// Karatsuba: 3 products; c0 = t0 - t1, c1 = t2 - t0 - t1
template <class A, class B>
BLS_HD auto l2_mul(const L2<A>& a, const L2<B>& b) {
  const auto t0 = lz_mul(a.c0, b.c0);
  const auto t1 = lz_mul(a.c1, b.c1);
  const auto t2 = lz_mul(lz_add(a.c0, a.c1), lz_add(b.c0, b.c1));
  return l2_join(lz_sub(t0, t1), lz_sub(lz_sub(t2, t0), t1));
}
// (a0 + a1)(a0 - a1), 2 a0 a1: two products, normalised output
template <class A>
BLS_HD auto l2_sqr(const L2<A>& a) {
  return l2_join(lz_mul(lz_add(a.c0, a.c1), lz_sub(a.c0, a.c1)), lz_mul(lz_dbl(a.c0), a.c1));
}
template <class A, class B>
BLS_HD auto l2_mul_fp(const L2<A>& a, const B& s) {
  return l2_join(lz_mul(a.c0, s), lz_mul(a.c1, s));
}

BLS_HD L2<LzIn> l2_from_fp2(const Fp2& a) { return L2<LzIn>{lz_from_fp(a.c0), lz_from_fp(a.c1)}; }
template <class A>
BLS_HD Fp2 l2_to_fp2(const L2<A>& a) {
  return Fp2{lz_to_fp(a.c0), lz_to_fp(a.c1)};
}

}  // namespace bls
