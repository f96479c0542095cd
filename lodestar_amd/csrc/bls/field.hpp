// BLS12-381 base-field tower for CDNA4 (gfx950): Fp, Fp2, Fp6, Fp12.
//
// Replaces the field arithmetic that the reference reaches through its
// un-vendored npm dependency @chainsafe/blst@0.2.4 -> supranational blst
// (yarn.lock:445-451); see SURVEY.md 2.2 items 1 and 6-7.
//
// Representation: Fp = 12 x 32-bit little-endian limbs in Montgomery form
// (R = 2^384).  One 381-bit element lives in 12 VGPRs of one lane; the VALU
// does the 32x32+64 multiply-adds (v_mad_u64_u32) of the CIOS product.  The
// modulus has 3 spare bits, so the "no-carry" CIOS variant applies (top limb of
// p < 2^31 - 1): the running 12-limb accumulator never needs a 13th word.
//
// Tower (same basis as the test oracle, oracle/bls_oracle.py):
//   Fp2  = Fp[u]  / (u^2 + 1)
//   Fp6  = Fp2[v] / (v^3 - xi),  xi = 1 + u
//   Fp12 = Fp6[w] / (w^2 - v)
// The Fp12 coefficient of w^k is (c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2)[k].
//
// Every function is __host__ __device__ so the same source is compiled for the
// GPU (the product) and for the CPU test harness tests/native/hostsim.cpp.
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BLS_HD __host__ __device__ __forceinline__
#define BLS_NOINLINE static __host__ __device__ __attribute__((noinline))
#else
#define BLS_HD static inline
#define BLS_NOINLINE static __attribute__((noinline))
#endif

#if defined(BLS_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
// Host-only operation counter (tests/native/hostsim.cpp): pins the algorithmic
// work model (Fp multiplications per stage) used for the roofline figure.
extern unsigned long long bls_fpm_counter;
#define BLS_COUNT_FPM() (++bls_fpm_counter)
#else
#define BLS_COUNT_FPM() ((void)0)
#endif

namespace bls {

struct Fp {
  uint32_t l[12];
};
struct Fp2 {
  Fp c0, c1;
};
struct Fp6 {
  Fp2 c0, c1, c2;
};
struct Fp12 {
  Fp6 c0, c1;
};

}  // namespace bls

#include "constants.hpp"

namespace bls {

BLS_HD uint32_t p_limb(int i) {
  const uint32_t t[12] = {BLS_P_LIMBS};
  return t[i];
}

// 32-bit add / subtract with carry.  With clang (hipcc, device and host) these are
// the carry builtins, which lower to v_add_co_u32 / v_addc_co_u32 / v_subb_co_u32
// chains on gfx950; the g++ build of the test harness uses 64-bit arithmetic.
#if defined(__clang__)
BLS_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  unsigned co;
  unsigned r = __builtin_addc(a, b, cin, &co);
  *cout = co;
  return r;
}
BLS_HD uint32_t subc32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  unsigned bo;
  unsigned r = __builtin_subc(a, b, bin, &bo);
  *bout = bo;
  return r;
}
#else
BLS_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  uint64_t t = (uint64_t)a + b + cin;
  *cout = (uint32_t)(t >> 32);
  return (uint32_t)t;
}
BLS_HD uint32_t subc32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  uint64_t t = (uint64_t)a - b - bin;
  *bout = (uint32_t)(t >> 63);
  return (uint32_t)t;
}
#endif

// ---------------------------------------------------------------------------
// Fp
// ---------------------------------------------------------------------------
BLS_HD Fp fp_zero() {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = 0;
  return r;
}

BLS_HD bool fp_is_zero(const Fp& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.l[i];
  return acc == 0;
}

BLS_HD bool fp_eq(const Fp& a, const Fp& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.l[i] ^ b.l[i];
  return acc == 0;
}

BLS_HD Fp fp_select(bool c, const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// a - p with borrow; returns borrow (1 if a < p)
BLS_HD uint32_t fp_sub_p(const Fp& a, Fp& d) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d.l[i] = subc32(a.l[i], p_limb(i), borrow, &borrow);
  return borrow;
}

#if defined(__HIPCC__)
}  // namespace bls
#include "carry_asm.hpp"
namespace bls {
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// gfx950: each chain is one inline-asm block (tools/gen_carry_asm.py)
BLS_HD Fp fp_reduce_once(const Fp& s) {
  const uint32_t pl[12] = {BLS_P_LIMBS};
  Fp r;
  asm_reduce12(r.l, s.l, pl);
  return r;
}

BLS_HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp s;
  asm_add12(s.l, a.l, b.l);  // a + b < 2p < 2^382: no carry out
  return fp_reduce_once(s);
}

BLS_HD Fp fp_sub(const Fp& a, const Fp& b) {
  const uint32_t pl[12] = {BLS_P_LIMBS};
  Fp d, r;
  uint32_t borrow = asm_sub12(d.l, a.l, b.l);
  asm_add12_masked(r.l, d.l, pl, 0u - borrow);  // a < b: add p back
  return r;
}

// Unreduced forms for a product's operands only (the 28-bit-digit product takes inputs
// < 3p, test_hostsim.py::test_fp_mul_d28_lazy): a + b < 2p and a + p - b in (0, 2p]
// for a, b < p
BLS_HD Fp fp_add_nr(const Fp& a, const Fp& b) {
  Fp s;
  asm_add12(s.l, a.l, b.l);
  return s;
}

BLS_HD Fp fp_sub_nr(const Fp& a, const Fp& b) {
  const uint32_t pl[12] = {BLS_P_LIMBS};
  Fp t, r;
  (void)asm_sub12(t.l, pl, b.l);  // p - b >= 1
  asm_add12(r.l, a.l, t.l);
  return r;
}

// a < 4p -> [0, 2p): one conditional subtraction of 2p (fp2_mul_s)
BLS_HD Fp fp_reduce_2p(const Fp& a) {
  const uint32_t pl2[12] = {BLS_2P_LIMBS};
  Fp r;
  asm_reduce12(r.l, a.l, pl2);
  return r;
}
#else
// Host build (CPU test harness and the CPU baseline under oracle/): the 12 x 32-bit
// little-endian limbs are the bytes of 6 x 64-bit little-endian words, so the CPU
// works on 64-bit words with unsigned __int128 carries (x86-64 host only).
static_assert(sizeof(Fp) == 48, "Fp is 6 x 64-bit words on the host");
static inline void fp_w_load(const Fp& a, uint64_t w[6]) { memcpy(w, a.l, 48); }
static inline Fp fp_w_store(const uint64_t w[6]) {
  Fp r;
  memcpy(r.l, w, 48);
  return r;
}
static const uint64_t BLS_P64[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                                    0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
#define BLS_NP0_64 0x89f3fffcfffcfffdull  // -p^-1 mod 2^64

// s - p when s >= p (s < 2p)
static inline void fp_w_reduce(uint64_t s[6]) {
  uint64_t d[6];
  unsigned __int128 br = 0;
  for (int i = 0; i < 6; ++i) {
    const unsigned __int128 t = (unsigned __int128)s[i] - BLS_P64[i] - (uint64_t)br;
    d[i] = (uint64_t)t;
    br = (t >> 64) & 1;
  }
  if (!br) memcpy(s, d, 48);
}

// Reduce a value < 2p to [0, p).
BLS_HD Fp fp_reduce_once(const Fp& a) {
  uint64_t s[6];
  fp_w_load(a, s);
  fp_w_reduce(s);
  return fp_w_store(s);
}

BLS_HD Fp fp_add(const Fp& a, const Fp& b) {
  uint64_t x[6], y[6];
  fp_w_load(a, x);
  fp_w_load(b, y);
  unsigned __int128 c = 0;
  for (int i = 0; i < 6; ++i) {
    c += (unsigned __int128)x[i] + y[i];
    x[i] = (uint64_t)c;
    c >>= 64;
  }
  fp_w_reduce(x);  // a + b < 2p < 2^382: no carry out
  return fp_w_store(x);
}

BLS_HD Fp fp_sub(const Fp& a, const Fp& b) {
  uint64_t x[6], y[6];
  fp_w_load(a, x);
  fp_w_load(b, y);
  unsigned __int128 br = 0;
  for (int i = 0; i < 6; ++i) {
    const unsigned __int128 t = (unsigned __int128)x[i] - y[i] - (uint64_t)br;
    x[i] = (uint64_t)t;
    br = (t >> 64) & 1;
  }
  if (br) {  // a < b: add p back
    unsigned __int128 c = 0;
    for (int i = 0; i < 6; ++i) {
      c += (unsigned __int128)x[i] + BLS_P64[i];
      x[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  return fp_w_store(x);
}

BLS_HD Fp fp_add_nr(const Fp& a, const Fp& b) {
  uint64_t x[6], y[6];
  fp_w_load(a, x);
  fp_w_load(b, y);
  unsigned __int128 c = 0;
  for (int i = 0; i < 6; ++i) {
    c += (unsigned __int128)x[i] + y[i];
    x[i] = (uint64_t)c;
    c >>= 64;
  }
  return fp_w_store(x);
}

BLS_HD Fp fp_sub_nr(const Fp& a, const Fp& b) {
  uint64_t x[6], y[6];
  fp_w_load(a, x);
  fp_w_load(b, y);
  unsigned __int128 br = 0, c = 0;
  for (int i = 0; i < 6; ++i) {  // y = p - b
    const unsigned __int128 t = (unsigned __int128)BLS_P64[i] - y[i] - (uint64_t)br;
    y[i] = (uint64_t)t;
    br = (t >> 64) & 1;
  }
  for (int i = 0; i < 6; ++i) {
    c += (unsigned __int128)x[i] + y[i];
    x[i] = (uint64_t)c;
    c >>= 64;
  }
  return fp_w_store(x);
}

BLS_HD Fp fp_reduce_2p(const Fp& a) {
  static const uint64_t P2[6] = {0x73fdffffffff5556ull, 0x3d57fffd62a7ffffull, 0xce61a541ed61ec48ull,
                                 0xc8ee9709e70a257eull, 0x96374f6c869759aeull, 0x340223d472ffcd34ull};
  uint64_t x[6], d[6];
  fp_w_load(a, x);
  unsigned __int128 br = 0;
  for (int i = 0; i < 6; ++i) {
    const unsigned __int128 t = (unsigned __int128)x[i] - P2[i] - (uint64_t)br;
    d[i] = (uint64_t)t;
    br = (t >> 64) & 1;
  }
  return fp_w_store(br ? x : d);
}
#endif

BLS_HD Fp fp_dbl(const Fp& a) { return fp_add(a, a); }

BLS_HD Fp fp_neg(const Fp& a) {
  Fp z = fp_zero();
  return fp_sub(z, a);
}

// a / 2 mod p
BLS_HD Fp fp_half(const Fp& a) {
  uint32_t mask = 0u - (a.l[0] & 1u);
  Fp s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) s.l[i] = addc32(a.l[i], p_limb(i) & mask, c, &c);
  Fp r;
#pragma unroll
  for (int i = 0; i < 11; ++i) r.l[i] = (s.l[i] >> 1) | (s.l[i + 1] << 31);
  r.l[11] = s.l[11] >> 1;  // a + p < 2^382: bit 384 never set
  return r;
}

// ---------------------------------------------------------------------------
// Montgomery product over 28-bit digits (the device product; portable, so the host
// harness checks it against the 64-bit product).  The 12 x 32-bit limbs are re-cut into
// 14 digits of 28 bits: a 28 x 28-bit product is < 2^56, so a 64-bit column absorbs all
// of its <= 28 products plus the carry from below without overflowing -- one
// v_mad_u64_u32 per product and no carry instruction, where 32-bit digits need a
// v_addc_co_u32 after every product.  196 (a*b) + 196 (m*p) products; the reduction takes
// 13 digits of 28 bits and one of 20 (R = 2^384, the Montgomery form of the whole
// library).  Inputs < 3p (< 2^383), output < 2p (9p^2/R + p < 2p); LAZY = false reduces
// the output to [0, p).
// ---------------------------------------------------------------------------
#define BLS_D28_MASK 0xFFFFFFFu
#define BLS_NP28 0xFFCFFFDu  // -p^-1 mod 2^28
BLS_HD uint32_t p28_digit(int k) {
  const uint32_t t[14] = {0xfffaaabu, 0xfefffffu, 0x3ffffb9u, 0xfffeb15u, 0x6241eabu, 0xa0f6b0fu, 0xf6730d2u,
                          0xf38512bu, 0x4774b84u, 0x4bacd76u, 0xba7b643u, 0xe69a4b1u, 0x1ea397fu, 0x001a011u};
  return t[k];
}

BLS_HD void fp_to_d28(const Fp& a, uint32_t d[14]) {
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int o = 28 * k, w = o >> 5, s = o & 31;
    const uint64_t pair = ((uint64_t)(w + 1 < 12 ? a.l[w + 1] : 0u) << 32) | a.l[w];
    d[k] = (uint32_t)(pair >> s) & BLS_D28_MASK;
  }
}

// t += a b (unsigned / signed 32 x 32 -> 64 multiply-add).  On the device each is one
// ordered v_mad_{u,i}64_i32: left to the compiler, the products were reassociated into
// trees held all at once (~230 VGPRs in fp2_mul_d28, which every caller must free)
#if defined(__HIP_DEVICE_COMPILE__)
#define BLS_D28_MAC(t, a, b)                                                        \
  do {                                                                              \
    uint64_t cc_;                                                                   \
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(t), "=&s"(cc_) : "v"(a), "v"(b)); \
  } while (0)
#define BLS_D28_MACS(t, a, b)                                                       \
  do {                                                                              \
    uint64_t cc_;                                                                   \
    asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(t), "=&s"(cc_) : "v"(a), "v"(b)); \
  } while (0)
// c is computed before any later asm block (the second half's multiply-adds): without it
// the compiler sank the first reduction below them, keeping both column sets live
#define BLS_PIN_FP(c)                                                                                \
  asm volatile("" ::"v"((c).l[0]), "v"((c).l[1]), "v"((c).l[2]), "v"((c).l[3]), "v"((c).l[4]),     \
               "v"((c).l[5]), "v"((c).l[6]), "v"((c).l[7]), "v"((c).l[8]), "v"((c).l[9]), "v"((c).l[10]), \
               "v"((c).l[11]))
#define BLS_D28_MACK(t, a, k)                                                                        \
  do {                                                                                               \
    uint64_t cc_;                                                                                    \
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(t), "=&s"(cc_) : "v"(a), "s"(k));        \
  } while (0)
#else
#define BLS_D28_MACK(t, a, k) ((t) += (uint64_t)(a) * (k))
#define BLS_PIN_FP(c) ((void)0)
#define BLS_D28_MAC(t, a, b) ((t) += (uint64_t)(a) * (b))
#define BLS_D28_MACS(t, a, b) ((t) = (uint64_t)((int64_t)(t) + (int64_t)(int32_t)(a) * (int64_t)(int32_t)(b)))
#endif

// t: the 27 columns of a 14 x 14-digit product; returns t / 2^384 mod p (< 2p)
// ORDERED: the m p multiply-adds as ordered asm (fp2_mul_d28, where the compiler otherwise
// holds them as product trees); the lone products keep the compiler's schedule (ordered,
// they measured ~10 % slower)
BLS_HD Fp fp_d28_tail(uint64_t t[27]);

template <bool ORDERED = false>
BLS_HD Fp fp_redc_d28(uint64_t t[27]) {
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const uint32_t m = ((uint32_t)t[i] * BLS_NP28) & BLS_D28_MASK;
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      if (ORDERED) BLS_D28_MACK(t[i + j], m, p28_digit(j));
      else t[i + j] += (uint64_t)m * p28_digit(j);
    }
    t[i + 1] += t[i] >> 28;  // column i is now 0 mod 2^28
  }
  {
    const uint32_t m = ((uint32_t)t[13] * BLS_NP28) & 0xFFFFFu;  // the last 20 bits
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      if (ORDERED) BLS_D28_MACK(t[13 + j], m, p28_digit(j));
      else t[13 + j] += (uint64_t)m * p28_digit(j);
    }
  }
  return fp_d28_tail(t);
}

// result = t[13] / 2^20 + sum_{k >= 14} t[k] 2^(8 + 28 (k - 14)) once columns 0..12 are
// 0 mod 2^28 and column 13 is 0 mod 2^20: normalise the digits from bit 8 on, then
// pack them into 32-bit limbs
BLS_HD Fp fp_d28_tail(uint64_t t[27]) {
  const uint64_t u = t[13] >> 20;
  t[14] += u >> 8;
#pragma unroll
  for (int k = 14; k < 26; ++k) {
    t[k + 1] += t[k] >> 28;
    t[k] &= BLS_D28_MASK;
  }
  Fp r;
  uint64_t acc = u & 0xFFu;
  int nb = 8, w = 0;
#pragma unroll
  for (int k = 14; k < 27; ++k) {
    acc |= t[k] << nb;  // t[26] < 2^38 lands at bit 24 of the last two limbs
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
  return r;
}

BLS_HD Fp fp_mul_d28_lazy(const Fp& a, const Fp& b) {
  uint32_t x[14], y[14];
  fp_to_d28(a, x);
  fp_to_d28(b, y);
  uint64_t t[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) t[i + j] += (uint64_t)x[i] * y[j];
  return fp_redc_d28(t);
}

// squaring: 14 squares + 91 cross products against doubled digits (< 2^29)
BLS_HD Fp fp_sqr_d28_lazy(const Fp& a) {
  uint32_t x[14], x2[14];
  fp_to_d28(a, x);
#pragma unroll
  for (int k = 0; k < 14; ++k) x2[k] = x[k] << 1;
  uint64_t t[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    t[2 * i] += (uint64_t)x[i] * x[i];
#pragma unroll
    for (int j = i + 1; j < 14; ++j) t[i + j] += (uint64_t)x2[i] * x[j];
  }
  return fp_redc_d28(t);
}

// Fp2 product with ONE Montgomery reduction per coefficient (lazy reduction), for
// canonical inputs (< p):
//   c0 = (a0 b0 - a1 b1) / R,  c1 = (a0 b1 + a1 b0) / R
// as 27-column 28-bit-digit products (4 x 196 digit products, 2 reductions of 196 --
// the same multiply-adds as three reduced products, without the third reduction, two
// operand conversions, the Karatsuba additions and the final subtractions).  c0's
// columns start from C2_COL, a multiple of p whose column k is at least the largest
// column k of a1 b1 for canonical digits (digits 0..12 < 2^28, digit 13 <= p >> 364),
// so every column stays >= 0 through the signed multiply-subtract of a1 b1 and the
// unsigned reduction applies: c0 value < p^2 + 2^762 -> output < 1.21 p; c1 < 2 p^2 ->
// < 1.42 p; one conditional subtraction each makes them canonical.  tests:
// test_hostsim.py::test_fp2_mul_lazy (C2_COL generated and checked there).
BLS_HD uint64_t c2_col(int k) {
  const uint64_t t[27] = {
      0x00ffffffe1cc48ddull, 0x01ffffffcec8d82dull, 0x02ffffffa9e42d7cull, 0x03ffffff8c5f88ffull, 0x04ffffff683c5c79ull,
      0x05ffffff4a84a061ull, 0x06ffffff2f404920ull, 0x07ffffff0efefe3bull, 0x08fffffee90b358cull, 0x09fffffec66cc7e1ull,
      0x0afffffea7af04abull, 0x0bfffffe892c9c2eull, 0x0cfffffe6149107bull, 0x0c0034009ffe581bull, 0x0b003400bffcbfe9ull,
      0x0a003400dffcbfe8ull, 0x09003400fffcbfe7ull, 0x080034011ffcbfe6ull, 0x070034013ffcbfe5ull, 0x060034015ffcbfe4ull,
      0x050034017ffcbfe3ull, 0x040034019ffcbfe2ull, 0x03003401bffcbfe1ull, 0x02003401dffcbfe0ull, 0x01003401fffcbfdfull,
      0x000034021ffcbfdeull, 0x00000002a4374121ull};
  return t[k];
}

// the device scheduler may not move instructions across (keeps the two halves of
// fp2_mul_d28 apart: interleaved they held ~250 VGPRs, which every caller must free)
#if defined(__HIP_DEVICE_COMPILE__)
#define BLS_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define BLS_SCHED_FENCE() ((void)0)
#endif

BLS_HD Fp2 fp2_mul_d28(const Fp& a0, const Fp& a1, const Fp& b0, const Fp& b1) {
  uint32_t x0[14], x1[14], y0[14], y1[14];
  fp_to_d28(a0, x0);
  fp_to_d28(a1, x1);
  fp_to_d28(b0, y0);
  fp_to_d28(b1, y1);
  uint64_t t[27];
  int32_t ny1[14];  // -b1's digits: a1 b1 leaves the columns by signed multiply-adds
#pragma unroll
  for (int j = 0; j < 14; ++j) ny1[j] = -(int32_t)y1[j];
#pragma unroll
  for (int k = 0; k < 27; ++k) t[k] = c2_col(k);
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      BLS_D28_MAC(t[i + j], x0[i], y0[j]);
      BLS_D28_MACS(t[i + j], x1[i], ny1[j]);
    }
  const Fp c0 = fp_reduce_once(fp_redc_d28<true>(t));
  BLS_PIN_FP(c0);
  BLS_SCHED_FENCE();
#pragma unroll
  for (int k = 0; k < 27; ++k) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      BLS_D28_MAC(t[i + j], x0[i], y1[j]);
      BLS_D28_MAC(t[i + j], x1[i], y0[j]);
    }
  return Fp2{c0, fp_reduce_once(fp_redc_d28<true>(t))};
}

// Fp2 square with one reduction per coefficient (canonical inputs): c0 = (a0^2 - a1^2)/R
// from the two symmetric squares (105 digit products each) on the C2_COL offset (a1^2's
// columns are bounded like a1 b1's), c1 = 2 a0 a1 / R from the doubled digits of a0
// (< 2^29).  tests: test_hostsim.py::test_fp2_mul_lazy.
BLS_HD Fp2 fp2_sqr_d28(const Fp& a0, const Fp& a1) {
  uint32_t x0[14], x1[14];
  fp_to_d28(a0, x0);
  fp_to_d28(a1, x1);
  uint64_t t[27];
  int32_t n1[14], n2[14];  // -a1 and -2 a1 digits
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    n1[j] = -(int32_t)x1[j];
    n2[j] = -(int32_t)(x1[j] << 1);
  }
#pragma unroll
  for (int k = 0; k < 27; ++k) t[k] = c2_col(k);
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    BLS_D28_MAC(t[2 * i], x0[i], x0[i]);
    BLS_D28_MACS(t[2 * i], x1[i], n1[i]);
#pragma unroll
    for (int j = i + 1; j < 14; ++j) {
      BLS_D28_MAC(t[i + j], x0[i] << 1, x0[j]);
      BLS_D28_MACS(t[i + j], x1[i], n2[j]);
    }
  }
  const Fp c0 = fp_reduce_once(fp_redc_d28<true>(t));
  BLS_PIN_FP(c0);
  BLS_SCHED_FENCE();
#pragma unroll
  for (int k = 0; k < 27; ++k) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) BLS_D28_MAC(t[i + j], x0[i] << 1, x1[j]);
  return Fp2{c0, fp_reduce_once(fp_redc_d28<true>(t))};
}

#if defined(__HIP_DEVICE_COMPILE__)
// gfx950: product-scanning (FIPS) Montgomery product.  Each 32x32 product is one
// v_mad_u64_u32 into a 64-bit column accumulator whose carry-out (VOP3B sdst) feeds
// a v_addc_co_u32 into the third accumulator word: 2 instructions per product,
// 288 products.  a*b and m*p products go to two accumulators (two dependency
// chains per column), merged once per column.
__device__ __forceinline__ void bls_mac(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
      "v_addc_co_u32 %1, %2, 0, %1, %2"
      : "+v"(lo), "+v"(hi), "=&s"(cc)
      : "v"(a), "v"(b));
}
__device__ __forceinline__ void bls_mac_s(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
      "v_addc_co_u32 %1, %2, 0, %1, %2"
      : "+v"(lo), "+v"(hi), "=&s"(cc)
      : "v"(a), "s"(b));
}
// one a*b product on chain 1 and one m*p product on chain 2, interleaved in one
// block (fewer inline-asm boundaries, two independent carry chains in flight)
__device__ __forceinline__ void bls_mac2(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b, uint64_t& lo2,
                                         uint32_t& hi2, uint32_t m, uint32_t p) {
  uint64_t c1, c2;
  asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"
      "v_mad_u64_u32 %2, %5, %8, %9, %2\n\t"
      "v_addc_co_u32 %1, %4, 0, %1, %4\n\t"
      "v_addc_co_u32 %3, %5, 0, %3, %5"
      : "+v"(lo), "+v"(hi), "+v"(lo2), "+v"(hi2), "=&s"(c1), "=&s"(c2)
      : "v"(a), "v"(b), "v"(m), "s"(p));
}

// Four independent multiply-accumulates (columns c0..c3) in one block: the four
// v_mad_u64_u32 issue back to back and each carry is consumed three instructions
// later, so the wave does not stall on the 64-bit multiply latency.
#define BLS_MAC4(L, H, k, x, y0, y1, y2, y3, YC)                                                       \
  do {                                                                                             \
    uint64_t c0_, c1_, c2_, c3_;                                                                   \
    asm("v_mad_u64_u32 %0, %8, %12, %13, %0\n\t"                                                  \
        "v_mad_u64_u32 %2, %9, %12, %14, %2\n\t"                                                  \
        "v_mad_u64_u32 %4, %10, %12, %15, %4\n\t"                                                 \
        "v_mad_u64_u32 %6, %11, %12, %16, %6\n\t"                                                 \
        "v_addc_co_u32 %1, %8, 0, %1, %8\n\t"                                                     \
        "v_addc_co_u32 %3, %9, 0, %3, %9\n\t"                                                     \
        "v_addc_co_u32 %5, %10, 0, %5, %10\n\t"                                                   \
        "v_addc_co_u32 %7, %11, 0, %7, %11"                                                        \
        : "+v"(L[k]), "+v"(H[k]), "+v"(L[k + 1]), "+v"(H[k + 1]), "+v"(L[k + 2]), "+v"(H[k + 2]),   \
          "+v"(L[k + 3]), "+v"(H[k + 3]), "=&s"(c0_), "=&s"(c1_), "=&s"(c2_), "=&s"(c3_)            \
        : "v"(x), YC(y0), YC(y1), YC(y2), YC(y3));                                                  \
  } while (0)

// 64-bit add of c into column (L, H): L += c, carry into H
__device__ __forceinline__ void bls_col_add(uint64_t& lo, uint32_t& hi, uint64_t c) {
  uint32_t l0 = (uint32_t)lo, l1 = (uint32_t)(lo >> 32);
  uint64_t cc;
  asm("v_add_co_u32 %0, %3, %0, %4\n\t"
      "v_addc_co_u32 %1, %3, %1, %5, %3\n\t"
      "v_addc_co_u32 %2, %3, 0, %2, %3"
      : "+v"(l0), "+v"(l1), "+v"(hi), "=&s"(cc)
      : "v"((uint32_t)c), "v"((uint32_t)(c >> 32)));
  lo = ((uint64_t)l1 << 32) | l0;
}

// gfx950 Montgomery product with column accumulators (separated operand scanning):
// the 144 a*b products fill 24 columns row by row, four independent columns per
// block; the reduction then adds m_i * p into columns i..i+11, where only
// m_i = col_i * (-p^-1) and the carry col_i >> 64-bit into col_{i+1} are on the
// dependency chain.  288 products, 2 instructions each.
// LAZY: inputs < 3p, output < 2p (no final subtraction; 9p^2/R + p < 2p since
// p < R/9.8) -- the cooperative interpreter's representation.  Otherwise canonical.
template <bool LAZY>
__device__ __forceinline__ Fp fp_mul_cols(const Fp& a, const Fp& b) {
  uint64_t L[24];
  uint32_t H[24];
#pragma unroll
  for (int k = 0; k < 24; ++k) {
    L[k] = 0;
    H[k] = 0;
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
#pragma unroll
    for (int j = 0; j < 12; j += 4) BLS_MAC4(L, H, i + j, a.l[i], b.l[j], b.l[j + 1], b.l[j + 2], b.l[j + 3], "v");
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint32_t m = (uint32_t)L[i] * BLS_NP0;
    BLS_MAC4(L, H, i, m, p_limb(0), p_limb(1), p_limb(2), p_limb(3), "s");
    // column i is now 0 mod 2^32: carry (col_i >> 32) into column i+1
    const uint64_t c = (L[i] >> 32) | ((uint64_t)H[i] << 32);
    bls_col_add(L[i + 1], H[i + 1], c);
    BLS_MAC4(L, H, i + 4, m, p_limb(4), p_limb(5), p_limb(6), p_limb(7), "s");
    BLS_MAC4(L, H, i + 8, m, p_limb(8), p_limb(9), p_limb(10), p_limb(11), "s");
  }
  Fp u;
#pragma unroll
  for (int k = 12; k < 23; ++k) {
    u.l[k - 12] = (uint32_t)L[k];
    const uint64_t c = (L[k] >> 32) | ((uint64_t)H[k] << 32);
    bls_col_add(L[k + 1], H[k + 1], c);
  }
  u.l[11] = (uint32_t)L[23];
  return LAZY ? u : fp_reduce_once(u);
}
// Montgomery square: 66 cross products (doubled) + 12 squares + the 144-product
// reduction = 222 multiply-adds instead of 288.
__device__ __forceinline__ Fp fp_sqr_cols(const Fp& a) {
  uint64_t L[24];
  uint32_t H[24];
#pragma unroll
  for (int k = 0; k < 24; ++k) {
    L[k] = 0;
    H[k] = 0;
  }
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    int j = i + 1;
#pragma unroll
    for (; j + 3 < 12; j += 4) BLS_MAC4(L, H, i + j, a.l[i], a.l[j], a.l[j + 1], a.l[j + 2], a.l[j + 3], "v");
#pragma unroll
    for (; j < 12; ++j) bls_mac(L[i + j], H[i + j], a.l[i], a.l[j]);
  }
#pragma unroll
  for (int k = 1; k < 23; ++k) {  // double the cross-product columns
    H[k] = (H[k] << 1) | (uint32_t)(L[k] >> 63);
    L[k] <<= 1;
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) bls_mac(L[2 * i], H[2 * i], a.l[i], a.l[i]);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint32_t m = (uint32_t)L[i] * BLS_NP0;
    BLS_MAC4(L, H, i, m, p_limb(0), p_limb(1), p_limb(2), p_limb(3), "s");
    const uint64_t c = (L[i] >> 32) | ((uint64_t)H[i] << 32);
    bls_col_add(L[i + 1], H[i + 1], c);
    BLS_MAC4(L, H, i + 4, m, p_limb(4), p_limb(5), p_limb(6), p_limb(7), "s");
    BLS_MAC4(L, H, i + 8, m, p_limb(8), p_limb(9), p_limb(10), p_limb(11), "s");
  }
  Fp u;
#pragma unroll
  for (int k = 12; k < 23; ++k) {
    u.l[k - 12] = (uint32_t)L[k];
    const uint64_t c = (L[k] >> 32) | ((uint64_t)H[k] << 32);
    bls_col_add(L[k + 1], H[k + 1], c);
  }
  u.l[11] = (uint32_t)L[23];
  return fp_reduce_once(u);
}
// BLS_FP_INLINE (a kernel TU that defines it before the includes): the product is
// inlined at every use instead of called -- no call boundary for the register
// allocator (k_chain's point chains keep their operands in registers)
#ifdef BLS_FP_INLINE
#define BLS_FP_MUL_ATTR static __device__ __forceinline__
#else
#define BLS_FP_MUL_ATTR BLS_NOINLINE
#endif
// BLS_FP_D28 (a kernel TU that defines it before the includes): the 28-bit-digit
// product (fp_mul_d28_lazy: ~580 VALU instructions instead of ~740 plus wait states,
// ~20 % lower latency per product on gfx950), out of line.  Opted into by k_pre, the
// cooperative interpreter kernels, k_chain, the Miller loops and the MSM; the other
// point-chain kernels keep the 32-bit-digit column product.  (Product-scanning and
// row-interleaved orders of the 28-bit product measured 3-8 % slower,
// profiles/r03_ab_product_order.json.)
#if !defined(BLS_FP_D28)
BLS_FP_MUL_ATTR Fp fp_sqr_dev(Fp a) { return fp_sqr_cols(a); }
__device__ __forceinline__ Fp fp_mul_inl(const Fp& a, const Fp& b) { return fp_mul_cols<false>(a, b); }
__device__ __forceinline__ Fp fp_mul_lazy(const Fp& a, const Fp& b) { return fp_mul_cols<true>(a, b); }
#else
BLS_FP_MUL_ATTR Fp fp_sqr_dev(Fp a) { return fp_reduce_once(fp_sqr_d28_lazy(a)); }
__device__ __forceinline__ Fp fp_mul_inl(const Fp& a, const Fp& b) { return fp_reduce_once(fp_mul_d28_lazy(a, b)); }
__device__ __forceinline__ Fp fp_mul_lazy(const Fp& a, const Fp& b) { return fp_mul_d28_lazy(a, b); }
#endif
// The out-of-line product takes its operands as 24 scalar words: passed as two Fp
// structs, the gfx950 calling convention hands the first one over by reference in
// private memory (the caller stores 48 B per lane to scratch, the callee loads them back
// at every product -- most of k_chain's ~380 KB of scratch traffic per set); scalars
// travel in v0-v23 and the result returns in v0-v11.
#define BLS_W12(x) uint32_t x##0, uint32_t x##1, uint32_t x##2, uint32_t x##3, uint32_t x##4, uint32_t x##5, \
                   uint32_t x##6, uint32_t x##7, uint32_t x##8, uint32_t x##9, uint32_t x##10, uint32_t x##11
#define BLS_FP_OF(x) Fp{{x##0, x##1, x##2, x##3, x##4, x##5, x##6, x##7, x##8, x##9, x##10, x##11}}
#define BLS_L12(v) (v).l[0], (v).l[1], (v).l[2], (v).l[3], (v).l[4], (v).l[5], (v).l[6], (v).l[7], (v).l[8], \
                   (v).l[9], (v).l[10], (v).l[11]
BLS_FP_MUL_ATTR Fp fp_mul_w(BLS_W12(a), BLS_W12(b)) { return fp_mul_inl(BLS_FP_OF(a), BLS_FP_OF(b)); }
BLS_FP_MUL_ATTR Fp fp_sqr_w(BLS_W12(a)) { return fp_sqr_dev(BLS_FP_OF(a)); }
__device__ __forceinline__ Fp fp_mul(const Fp& a, const Fp& b) { return fp_mul_w(BLS_L12(a), BLS_L12(b)); }
#else
// Host build: Montgomery product a*b/R mod p (R = 2^384) over 6 x 64-bit words,
// separated operand scanning (the 36 partial products of a*b first, then the word-by-
// word reduction), unsigned __int128 products.  Inputs < 2p (fp2_mul / fp2_sqr pass
// unreduced sums, fp_add_nr), output < p.
BLS_HD Fp fp_mul(const Fp& a, const Fp& b) {
  BLS_COUNT_FPM();
  typedef unsigned __int128 u128;
  uint64_t x[6], y[6], t[13];
  fp_w_load(a, x);
  fp_w_load(b, y);
  for (int k = 0; k < 13; ++k) t[k] = 0;
  for (int i = 0; i < 6; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 6; ++j) {
      const u128 v = (u128)x[i] * y[j] + t[i + j] + c;
      t[i + j] = (uint64_t)v;
      c = (uint64_t)(v >> 64);
    }
    t[i + 6] = c;
  }
  for (int i = 0; i < 6; ++i) {
    const uint64_t m = t[i] * BLS_NP0_64;
    uint64_t c = 0;
    for (int j = 0; j < 6; ++j) {
      const u128 v = (u128)m * BLS_P64[j] + t[i + j] + c;
      t[i + j] = (uint64_t)v;
      c = (uint64_t)(v >> 64);
    }
    for (int k = i + 6; k < 13 && c; ++k) {
      const u128 v = (u128)t[k] + c;
      t[k] = (uint64_t)v;
      c = (uint64_t)(v >> 64);
    }
  }
  fp_w_reduce(t + 6);  // t < 2p
  return fp_w_store(t + 6);
}
BLS_HD Fp fp_mul_inl(const Fp& a, const Fp& b) { return fp_mul(a, b); }
BLS_HD Fp fp_mul_lazy(const Fp& a, const Fp& b) { return fp_mul(a, b); }
#endif

#if defined(__HIP_DEVICE_COMPILE__)
BLS_HD Fp fp_sqr(const Fp& a) { return fp_sqr_w(BLS_L12(a)); }
#else
BLS_HD Fp fp_sqr(const Fp& a) { return fp_mul(a, a); }
#endif

BLS_HD Fp fp_to_mont(const Fp& a) { return fp_mul(a, c_r2()); }

BLS_HD Fp fp_from_mont(const Fp& a) {
  Fp one = fp_zero();
  one.l[0] = 1;
  return fp_mul(a, one);
}

}  // namespace bls
#include "lazy28.hpp"
namespace bls {

// a^e for an exponent given as a limb accessor (wave-uniform, MSB first).
// BLS_LAZY_POW (every device build; the CPU test harness and the work model define it,
// the CPU baseline does not): the chain runs in the lazy 28-bit-digit form
// (lazy28.hpp lz_pow_const: no limb re-cut, pack or final subtraction per product).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(BLS_LAZY_POW)
#define BLS_LAZY_POW 1
#endif
#ifdef BLS_LAZY_POW
template <uint32_t (*E)(int), int BITS>
BLS_HD Fp fp_pow_const(const Fp& a) {
  return lz_pow_const<E, BITS>(a);
}
#else
template <uint32_t (*E)(int), int BITS>
BLS_HD Fp fp_pow_const(const Fp& a) {
  // sliding window of width 4 over the fixed exponent, odd powers a, a^3, .., a^15
  Fp tab[8];
  tab[0] = a;
  const Fp a2 = fp_sqr(a);
  for (int k = 1; k < 8; ++k) tab[k] = fp_mul(tab[k - 1], a2);
  Fp r = a;
  bool started = false;
  int i = BITS - 1;
  while (i >= 0) {
    if (!((E(i >> 5) >> (i & 31)) & 1u)) {
      r = fp_sqr(r);
      --i;
      continue;
    }
    int j = i - 3 < 0 ? 0 : i - 3;
    while (!((E(j >> 5) >> (j & 31)) & 1u)) ++j;
    uint32_t val = 0;
    for (int k = i; k >= j; --k) {
      val = (val << 1) | ((E(k >> 5) >> (k & 31)) & 1u);
      if (started) r = fp_sqr(r);
    }
    r = started ? fp_mul(r, tab[val >> 1]) : tab[val >> 1];
    started = true;
    i = j - 1;
  }
  return r;
}
#endif

BLS_HD Fp fp_inv(const Fp& a) { return fp_pow_const<e_p_minus_2, E_P_MINUS_2_BITS>(a); }

// ---------------------------------------------------------------------------
// Fp inversion without Fermat's ~450 dependent Montgomery products (fp_inv_gcd below).
// ---------------------------------------------------------------------------
BLS_HD bool big_is_one(const Fp& a) {
  uint32_t acc = a.l[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 12; ++i) acc |= a.l[i];
  return acc == 0;
}

BLS_HD void big_shr1(Fp& a) {
#pragma unroll
  for (int i = 0; i < 11; ++i) a.l[i] = (a.l[i] >> 1) | (a.l[i + 1] << 31);
  a.l[11] >>= 1;
}

// a >= b (plain 384-bit)
BLS_HD bool big_geq(const Fp& a, const Fp& b) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint64_t t = (uint64_t)a.l[i] - b.l[i] - borrow;
    borrow = (uint32_t)(t >> 63);
  }
  return borrow == 0;
}

BLS_HD void big_sub(Fp& a, const Fp& b) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint64_t t = (uint64_t)a.l[i] - b.l[i] - borrow;
    a.l[i] = (uint32_t)t;
    borrow = (uint32_t)(t >> 63);
  }
}

// Signed 416-bit integers (13 two's-complement 32-bit limbs) for the inversion below.
struct Big13 {
  uint32_t l[13];
};

// (u x + v y) >> 30 for 30-divstep matrix entries |u| + |v| <= 2^30 (the low 30 bits
// of u x + v y are zero by construction)
BLS_HD Big13 big13_lin_shr30(const Big13& x, const Big13& y, int32_t u, int32_t v) {
  uint32_t t[13];
  int64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int64_t xi = i < 12 ? (int64_t)x.l[i] : (int64_t)(int32_t)x.l[i];
    const int64_t yi = i < 12 ? (int64_t)y.l[i] : (int64_t)(int32_t)y.l[i];
    const int64_t s = carry + (int64_t)u * xi + (int64_t)v * yi;  // |s| < 2^63
    t[i] = (uint32_t)s;
    carry = s >> 32;
  }
  Big13 r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = (t[i] >> 30) | (t[i + 1] << 2);
  r.l[12] = (uint32_t)((int32_t)t[12] >> 30);
  return r;
}

// (u d + v e) / 2^30 mod p for |d|, |e| < p: add k p with k = t * (-1/p) mod 2^30 so the
// low 30 bits vanish, shift; the result lies in (-2p, 2p) and is brought back to (-p, p)
BLS_HD Big13 big13_lin_modp_shr30(const Big13& d, const Big13& e, int32_t u, int32_t v) {
  uint32_t t[13];
  int64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int64_t di = i < 12 ? (int64_t)d.l[i] : (int64_t)(int32_t)d.l[i];
    const int64_t ei = i < 12 ? (int64_t)e.l[i] : (int64_t)(int32_t)e.l[i];
    const int64_t s = carry + (int64_t)u * di + (int64_t)v * ei;
    t[i] = (uint32_t)s;
    carry = s >> 32;
  }
  const uint32_t k = (t[0] * BLS_NP0) & 0x3fffffffu;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint64_t s = (uint64_t)t[i] + (uint64_t)k * p_limb(i) + c;
    t[i] = (uint32_t)s;
    c = s >> 32;
  }
  t[12] += (uint32_t)c;
  Big13 r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = (t[i] >> 30) | (t[i + 1] << 2);
  r.l[12] = (uint32_t)((int32_t)t[12] >> 30);
  // (-2p, 2p) -> (-p, p): subtract p when >= p, add p when < -p
  Big13 m;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const uint64_t s = (uint64_t)r.l[i] - (i < 12 ? p_limb(i) : 0u) - borrow;
    m.l[i] = (uint32_t)s;
    borrow = (uint32_t)(s >> 63);
  }
  const bool ge_p = (int32_t)m.l[12] >= 0;
  uint32_t cc = 0;
  Big13 q;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const uint64_t s = (uint64_t)r.l[i] + (i < 12 ? p_limb(i) : 0u) + cc;
    q.l[i] = (uint32_t)s;
    cc = (uint32_t)(s >> 32);
  }
  const bool lt_mp = (int32_t)q.l[12] < 0;  // r + p < 0
#pragma unroll
  for (int i = 0; i < 13; ++i) r.l[i] = ge_p ? m.l[i] : (lt_mp ? q.l[i] : r.l[i]);
  return r;
}

// Fp inversion by Bernstein-Yang "safegcd" divsteps, 30 per matrix: 37 rounds
// (1110 divsteps >= the (49 d + 80) / 17 = 1103 bound for d = 381-bit operands), each
// 30 branch-free divsteps on the low words, then the 416-bit updates of (f, g) and of
// the Bezout pair (d, e) mod p.  Fixed work (no data-dependent loop length, no lane
// divergence), ~40k instructions instead of the binary GCD's ~760 divergent shift
// steps.  In: a in Montgomery form (aR, canonical).  Out: a^-1 R; 0 -> 0.
BLS_NOINLINE Fp fp_inv_gcd(Fp a) {
  if (fp_is_zero(a)) return fp_zero();
  Big13 f, g, d, e;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    f.l[i] = p_limb(i);
    g.l[i] = a.l[i];
    d.l[i] = 0;
    e.l[i] = 0;
  }
  f.l[12] = g.l[12] = d.l[12] = e.l[12] = 0;
  e.l[0] = 1;
  int32_t delta = 1;
  for (int round = 0; round < 37; ++round) {
    uint32_t fl = f.l[0], gl = g.l[0];
    int32_t u = 1, v = 0, q = 0, r = 1;  // rows of the transition matrix x 2^steps
    for (int s = 0; s < 30; ++s) {
      const bool godd = (gl & 1u) != 0;
      const bool swap = godd && delta > 0;
      // swap: (f, g) <- (g, -f) (then the odd-g step below gives (g - f) / 2)
      const uint32_t nfl = swap ? gl : fl, ngl = swap ? (0u - fl) : gl;
      const int32_t nu = swap ? q : u, nv = swap ? r : v, nq = swap ? -u : q, nr = swap ? -v : r;
      delta = swap ? -delta : delta;
      fl = nfl;
      gl = ngl;
      u = nu;
      v = nv;
      q = nq;
      r = nr;
      gl += godd ? fl : 0u;  // odd g: g <- g + f
      q += godd ? u : 0;
      r += godd ? v : 0;
      gl >>= 1;
      u *= 2;
      v *= 2;
      delta += 1;
    }
    // 2^30 (f', g') = (u f + v g, q f + r g); (d', e') likewise, divided by 2^30 mod p
    const Big13 f2 = big13_lin_shr30(f, g, u, v);
    const Big13 g2 = big13_lin_shr30(f, g, q, r);
    const Big13 d2 = big13_lin_modp_shr30(d, e, u, v);
    const Big13 e2 = big13_lin_modp_shr30(d, e, q, r);
    f = f2;
    g = g2;
    d = d2;
    e = e2;
  }
  // g = 0, f = +-1: a^-1 = sign(f) d (mod p), d in (-p, p)
  const bool fneg = (int32_t)f.l[12] < 0;
  Big13 x;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {  // x = fneg ? -d : d
    const uint64_t s = (uint64_t)0 - d.l[i] - borrow;
    x.l[i] = fneg ? (uint32_t)s : d.l[i];
    borrow = (uint32_t)(s >> 63);
  }
  const bool xneg = (int32_t)x.l[12] < 0;
  Fp inv;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {  // into [0, p)
    const uint64_t s = (uint64_t)x.l[i] + (xneg ? p_limb(i) : 0u) + c;
    inv.l[i] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  return fp_mul(inv, c_r3());  // (aR)^-1 R^3 / R = a^-1 R
}


// Is the (plain, non-Montgomery) value a > (p-1)/2 ?  (ZCash "lexicographically largest")
BLS_HD bool fp_plain_gt_half(const Fp& a) {
  const uint32_t h[12] = {BLS_HALF_P_LIMBS};
  // compute h - a; borrow => a > h
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint64_t t = (uint64_t)h[i] - a.l[i] - borrow;
    borrow = (uint32_t)(t >> 63);
  }
  return borrow != 0;
}

BLS_HD bool fp_lex_largest(const Fp& a_mont) { return fp_plain_gt_half(fp_from_mont(a_mont)); }

// plain a < p ?
BLS_HD bool fp_plain_is_canonical(const Fp& a) {
  Fp d;
  return fp_sub_p(a, d) != 0;
}

// 48 big-endian bytes -> plain limbs (no reduction)
BLS_HD Fp fp_from_be48(const uint8_t* b) {
  Fp r;
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    const uint8_t* q = b + 44 - 4 * k;
    r.l[k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  return r;
}

BLS_HD void fp_to_be48(const Fp& a, uint8_t* b) {
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    uint8_t* q = b + 44 - 4 * k;
    q[0] = (uint8_t)(a.l[k] >> 24);
    q[1] = (uint8_t)(a.l[k] >> 16);
    q[2] = (uint8_t)(a.l[k] >> 8);
    q[3] = (uint8_t)a.l[k];
  }
}

// Fp square root (p = 3 mod 4): returns true and r with r^2 = a if a is a square.
BLS_HD bool fp_sqrt(const Fp& a, Fp& r) {
  r = fp_pow_const<e_p_plus_1_div_4, E_P_PLUS_1_DIV_4_BITS>(a);
  return fp_eq(fp_sqr(r), a);
}

// ---------------------------------------------------------------------------
// Fp2 = Fp[u]/(u^2+1)
// ---------------------------------------------------------------------------
BLS_HD Fp2 fp2_zero() { return Fp2{fp_zero(), fp_zero()}; }
BLS_HD Fp2 fp2_one() { return Fp2{c_one(), fp_zero()}; }
BLS_HD bool fp2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
BLS_HD bool fp2_eq(const Fp2& a, const Fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
BLS_HD Fp2 fp2_select(bool c, const Fp2& a, const Fp2& b) {
  return Fp2{fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)};
}
BLS_HD Fp2 fp2_add(const Fp2& a, const Fp2& b) { return Fp2{fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
BLS_HD Fp2 fp2_sub(const Fp2& a, const Fp2& b) { return Fp2{fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
BLS_HD Fp2 fp2_dbl(const Fp2& a) { return Fp2{fp_dbl(a.c0), fp_dbl(a.c1)}; }
BLS_HD Fp2 fp2_neg(const Fp2& a) { return Fp2{fp_neg(a.c0), fp_neg(a.c1)}; }
BLS_HD Fp2 fp2_conj(const Fp2& a) { return Fp2{a.c0, fp_neg(a.c1)}; }
BLS_HD Fp2 fp2_half(const Fp2& a) { return Fp2{fp_half(a.c0), fp_half(a.c1)}; }
BLS_HD Fp2 fp2_mul_fp(const Fp2& a, const Fp& b) { return Fp2{fp_mul(a.c0, b), fp_mul(a.c1, b)}; }

// Karatsuba with unreduced pre-additions (operands < 2p; reduced ones measured 3 % slower
// at the plateau, profiles/r03_ab_fp2_preadd.json)
BLS_HD Fp2 fp2_mul(const Fp2& a, const Fp2& b) {
  Fp t0 = fp_mul(a.c0, b.c0);
  Fp t1 = fp_mul(a.c1, b.c1);
  Fp t2 = fp_mul(fp_add_nr(a.c0, a.c1), fp_add_nr(b.c0, b.c1));  // operands < 2p
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}

// the same product for operands whose coefficients are unreduced sums (< 2p each,
// fp2_add_nr of canonical values): a0 b0 and a1 b1 < 4p^2, and (a0 + a1) brought back
// under 2p times (b0 + b1) < 4p is < 8p^2 < 2^384 p, inside the Montgomery product's
// input bound (its output < 2p, then canonical); output canonical.  Saves the four
// reductions of the pre-additions for one here (tests: test_hostsim.py::test_fp2_mul_s)
BLS_HD Fp2 fp2_mul_s(const Fp2& a, const Fp2& b) {
  Fp t0 = fp_mul(a.c0, b.c0);
  Fp t1 = fp_mul(a.c1, b.c1);
  Fp t2 = fp_mul(fp_reduce_2p(fp_add_nr(a.c0, a.c1)), fp_add_nr(b.c0, b.c1));
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
BLS_HD Fp2 fp2_add_nr(const Fp2& a, const Fp2& b) { return Fp2{fp_add_nr(a.c0, b.c0), fp_add_nr(a.c1, b.c1)}; }

BLS_HD Fp2 fp2_sqr(const Fp2& a) {
  Fp t0 = fp_mul(fp_add_nr(a.c0, a.c1), fp_sub_nr(a.c0, a.c1));  // operands < 2p
  Fp t1 = fp_mul(fp_add_nr(a.c0, a.c0), a.c1);                   // 2 a0 a1
  return Fp2{t0, t1};
}

// a * (1 + u)
BLS_HD Fp2 fp2_mul_xi(const Fp2& a) { return Fp2{fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

BLS_HD Fp2 fp2_inv(const Fp2& a) {
  Fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  Fp ni = fp_inv(n);
  return Fp2{fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}

// RFC 9380 sgn0 for m = 2 (on Montgomery inputs)
BLS_HD uint32_t fp2_sgn0(const Fp2& a) {
  Fp p0 = fp_from_mont(a.c0);
  Fp p1 = fp_from_mont(a.c1);
  uint32_t s0 = p0.l[0] & 1u;
  uint32_t z0 = fp_is_zero(p0) ? 1u : 0u;
  uint32_t s1 = p1.l[0] & 1u;
  return s0 | (z0 & s1);
}

// ZCash serialization sign bit for G2 y (compare c1 first, c0 if c1 == 0)
BLS_HD bool fp2_lex_largest(const Fp2& a) {
  Fp p1 = fp_from_mont(a.c1);
  if (!fp_is_zero(p1)) return fp_plain_gt_half(p1);
  return fp_plain_gt_half(fp_from_mont(a.c0));
}

// Square root in Fp2 via the norm (two Fp exponentiations).  Returns false iff a
// is not a square.  For a square a the result satisfies r^2 = a (either root).
//   alpha = a0^2 + a1^2, gamma = sqrt(alpha)        (a square <=> alpha square)
//   d = (a0 + gamma)/2, t = d^((p-3)/4)
//   d square:      r = d t + (a1 t / 2) u
//   d non-square:  r = (a1 t / 2) - (d t) u
BLS_HD bool fp2_sqrt(const Fp2& a, Fp2& r) {
  if (fp_is_zero(a.c1)) {
    Fp s;
    if (fp_sqrt(a.c0, s)) {
      r = Fp2{s, fp_zero()};
      return true;
    }
    // a0 non-square in Fp: sqrt(a0) = u * sqrt(-a0) since -1 is a non-square
    fp_sqrt(fp_neg(a.c0), s);
    r = Fp2{fp_zero(), s};
    return true;
  }
  Fp alpha = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  Fp gamma;
  if (!fp_sqrt(alpha, gamma)) return false;
  Fp d = fp_half(fp_add(a.c0, gamma));
  Fp t = fp_pow_const<e_p_minus_3_div_4, E_P_MINUS_3_DIV_4_BITS>(d);
  Fp dt = fp_mul(d, t);
  Fp a1t2 = fp_half(fp_mul(a.c1, t));
  if (fp_eq(fp_sqr(dt), d)) {
    r = Fp2{dt, a1t2};
  } else {
    r = Fp2{a1t2, fp_neg(dt)};
  }
  return true;
}

// ---------------------------------------------------------------------------
// Fp6 = Fp2[v]/(v^3 - xi)
// ---------------------------------------------------------------------------
BLS_HD Fp6 fp6_zero() { return Fp6{fp2_zero(), fp2_zero(), fp2_zero()}; }
BLS_HD Fp6 fp6_one() { return Fp6{fp2_one(), fp2_zero(), fp2_zero()}; }
BLS_HD Fp6 fp6_add(const Fp6& a, const Fp6& b) {
  return Fp6{fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)};
}
BLS_HD Fp6 fp6_sub(const Fp6& a, const Fp6& b) {
  return Fp6{fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)};
}
BLS_HD Fp6 fp6_neg(const Fp6& a) { return Fp6{fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
BLS_HD bool fp6_eq(const Fp6& a, const Fp6& b) {
  return fp2_eq(a.c0, b.c0) && fp2_eq(a.c1, b.c1) && fp2_eq(a.c2, b.c2);
}
// a * v
BLS_HD Fp6 fp6_mul_v(const Fp6& a) { return Fp6{fp2_mul_xi(a.c2), a.c0, a.c1}; }

BLS_HD Fp6 fp6_mul(const Fp6& a, const Fp6& b) {
  Fp2 t0 = fp2_mul(a.c0, b.c0);
  Fp2 t1 = fp2_mul(a.c1, b.c1);
  Fp2 t2 = fp2_mul(a.c2, b.c2);
  // (the Karatsuba pre-additions stay unreduced: fp2_mul_s)
  Fp2 c0 = fp2_sub(fp2_sub(fp2_mul_s(fp2_add_nr(a.c1, a.c2), fp2_add_nr(b.c1, b.c2)), t1), t2);
  c0 = fp2_add(fp2_mul_xi(c0), t0);
  Fp2 c1 = fp2_sub(fp2_sub(fp2_mul_s(fp2_add_nr(a.c0, a.c1), fp2_add_nr(b.c0, b.c1)), t0), t1);
  c1 = fp2_add(c1, fp2_mul_xi(t2));
  Fp2 c2 = fp2_sub(fp2_sub(fp2_mul_s(fp2_add_nr(a.c0, a.c2), fp2_add_nr(b.c0, b.c2)), t0), t2);
  c2 = fp2_add(c2, t1);
  return Fp6{c0, c1, c2};
}

BLS_HD Fp6 fp6_sqr(const Fp6& a) { return fp6_mul(a, a); }

// a * (d0 + d1 v)
BLS_HD Fp6 fp6_mul_01(const Fp6& a, const Fp2& d0, const Fp2& d1) {
  Fp2 a0d0 = fp2_mul(a.c0, d0);
  Fp2 a1d1 = fp2_mul(a.c1, d1);
  Fp2 c0 = fp2_add(a0d0, fp2_mul_xi(fp2_mul(a.c2, d1)));
  Fp2 c1 = fp2_sub(fp2_sub(fp2_mul_s(fp2_add_nr(a.c0, a.c1), fp2_add_nr(d0, d1)), a0d0), a1d1);
  Fp2 c2 = fp2_add(a1d1, fp2_mul(a.c2, d0));
  return Fp6{c0, c1, c2};
}

// a * (d1 v)
BLS_HD Fp6 fp6_mul_1(const Fp6& a, const Fp2& d1) {
  return Fp6{fp2_mul_xi(fp2_mul(a.c2, d1)), fp2_mul(a.c0, d1), fp2_mul(a.c1, d1)};
}

BLS_HD Fp6 fp6_inv(const Fp6& a) {
  Fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  Fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  Fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  Fp2 n = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  Fp2 ni = fp2_inv(n);
  return Fp6{fp2_mul(t0, ni), fp2_mul(t1, ni), fp2_mul(t2, ni)};
}

// ---------------------------------------------------------------------------
// Fp12 = Fp6[w]/(w^2 - v)
// ---------------------------------------------------------------------------
BLS_HD Fp12 fp12_one() { return Fp12{fp6_one(), fp6_zero()}; }
BLS_HD bool fp12_eq(const Fp12& a, const Fp12& b) { return fp6_eq(a.c0, b.c0) && fp6_eq(a.c1, b.c1); }
BLS_HD bool fp12_is_one(const Fp12& a) { return fp12_eq(a, fp12_one()); }
BLS_HD Fp12 fp12_conj(const Fp12& a) { return Fp12{a.c0, fp6_neg(a.c1)}; }

BLS_NOINLINE Fp12 fp12_mul(const Fp12& a, const Fp12& b) {
  Fp6 t0 = fp6_mul(a.c0, b.c0);
  Fp6 t1 = fp6_mul(a.c1, b.c1);
  Fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), t0), t1);
  Fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return Fp12{c0, c1};
}

// complex squaring: (A + Bw)^2 = (A^2 + v B^2) + 2AB w
BLS_NOINLINE Fp12 fp12_sqr(const Fp12& a) {
  Fp6 ab = fp6_mul(a.c0, a.c1);
  Fp6 s = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  Fp6 c0 = fp6_sub(fp6_sub(s, ab), fp6_mul_v(ab));
  Fp6 c1 = fp6_add(ab, ab);
  return Fp12{c0, c1};
}

// f * (l0 + l2 w^2 + l3 w^3): the M-twist line shape (arkworks mul_by_014)
BLS_NOINLINE Fp12 fp12_mul_line(const Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3) {
  Fp6 aa = fp6_mul_01(f.c0, l0, l2);
  Fp6 bb = fp6_mul_1(f.c1, l3);
  Fp6 c1 = fp6_sub(fp6_sub(fp6_mul_01(fp6_add(f.c0, f.c1), l0, fp2_add(l2, l3)), aa), bb);
  Fp6 c0 = fp6_add(aa, fp6_mul_v(bb));
  return Fp12{c0, c1};
}

// f * L * M for two lines of the mul_by_014 shape (l0 + l2 w^2 + l3 w^3): the product of
// the lines first (6 Fp2 products, w^6 = xi, no w^1 term: P.c0 = (A0, A2, A4), P.c1 =
// (0, A3, A5)), then f * P by Karatsuba over Fp6 (6 + 5 + 6): 23 Fp2 products instead of
// the 26 of two fp12_mul_line calls.  Same value as fp12_mul_line(fp12_mul_line(f, L), M)
// (test_hostsim.py::test_fp12_mul_line2); the shared-f Miller loops (kernels/k_mlq.hip).
BLS_HD Fp12 fp12_mul_line2(const Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3, const Fp2& m0,
                           const Fp2& m2, const Fp2& m3) {
  const Fp2 m00 = fp2_mul(l0, m0), m22 = fp2_mul(l2, m2), m33 = fp2_mul(l3, m3);
  const Fp2 a0 = fp2_add(m00, fp2_mul_xi(m33));
  const Fp2 a2 = fp2_sub(fp2_sub(fp2_mul_s(fp2_add_nr(l0, l2), fp2_add_nr(m0, m2)), m00), m22);
  const Fp2 a3 = fp2_sub(fp2_sub(fp2_mul_s(fp2_add_nr(l0, l3), fp2_add_nr(m0, m3)), m00), m33);
  const Fp2 a5 = fp2_sub(fp2_sub(fp2_mul_s(fp2_add_nr(l2, l3), fp2_add_nr(m2, m3)), m22), m33);
  const Fp6 p0 = Fp6{a0, a2, m22};
  const Fp6 t0 = fp6_mul(f.c0, p0);
  const Fp6 t1 = fp6_mul_v(fp6_mul_01(f.c1, a3, a5));  // f.c1 * (a3 v + a5 v^2)
  const Fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(f.c0, f.c1), Fp6{a0, fp2_add(a2, a3), fp2_add(m22, a5)}), t0), t1);
  return Fp12{fp6_add(t0, fp6_mul_v(t1)), c1};
}

// One f over two lanes (kernels/k_mlq.hip k_mlf2): each half computes one part of the
// products (_prod), the halves swap their parts, and both finish alike (_join).  Host-
// tested against fp12_sqr / fp12_mul_line with both halves run one after the other
// (test_hostsim.py::test_fp12_pair_halves).
//   (A + B w)^2 = (s - ab - v ab) + 2 ab w: half 0 ab = A B, half 1 s = (A + B)(A + v B)
BLS_HD Fp6 fp12_sqr_half_prod(const Fp12& a, bool h) {
  return fp6_mul(h ? fp6_add(a.c0, a.c1) : a.c0, h ? fp6_add(a.c0, fp6_mul_v(a.c1)) : a.c1);
}
BLS_HD Fp12 fp12_sqr_half_join(const Fp6& own, const Fp6& other, bool h) {
  const Fp6 ab = h ? other : own, s = h ? own : other;
  return Fp12{fp6_sub(fp6_sub(s, ab), fp6_mul_v(ab)), fp6_add(ab, ab)};
}
//   f (l0 + l2 w^2 + l3 w^3): half 0 aa = f.c0 (l0 + l2 v), half 1 t = (f.c0 + f.c1)(l0 +
//   (l2 + l3) v); bb = f.c1 l3 v = (xi c2 l3, c0 l3, c1 l3) of f.c1: half 0 c2 l3, half 1
//   c0 l3, both c1 l3 (q)
struct LineHalf {
  Fp6 m;
  Fp2 p, q;
};
BLS_HD LineHalf fp12_line_half_prod(const Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3, bool h) {
  LineHalf r;
  r.m = fp6_mul_01(h ? fp6_add(f.c0, f.c1) : f.c0, l0, h ? fp2_add(l2, l3) : l2);
  r.p = fp2_mul(h ? f.c1.c0 : f.c1.c2, l3);
  r.q = fp2_mul(f.c1.c1, l3);
  return r;
}
BLS_HD Fp12 fp12_line_half_join(const LineHalf& own, const Fp6& m_other, const Fp2& p_other, bool h) {
  const Fp6 aa = h ? m_other : own.m, t = h ? own.m : m_other;
  const Fp6 bb = Fp6{fp2_mul_xi(h ? p_other : own.p), h ? own.p : p_other, own.q};
  return Fp12{fp6_add(aa, fp6_mul_v(bb)), fp6_sub(fp6_sub(t, aa), bb)};
}

BLS_HD Fp12 fp12_inv(const Fp12& a) {
  Fp6 n = fp6_sub(fp6_sqr(a.c0), fp6_mul_v(fp6_sqr(a.c1)));
  Fp6 ni = fp6_inv(n);
  return Fp12{fp6_mul(a.c0, ni), fp6_neg(fp6_mul(a.c1, ni))};
}

// f^p: coefficient k of w^k -> conj(c_k) * xi^(k(p-1)/6)
BLS_HD Fp12 fp12_frob(const Fp12& a) {
  Fp12 r;
  r.c0.c0 = fp2_conj(a.c0.c0);                          // w^0
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), c_frob1_1());    // w^1
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), c_frob1_2());    // w^2
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), c_frob1_3());    // w^3
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), c_frob1_4());    // w^4
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), c_frob1_5());    // w^5
  return r;
}

// f^(p^2): coefficient k -> c_k * xi^(k(p^2-1)/6)  (an Fp scalar)
BLS_HD Fp12 fp12_frob2(const Fp12& a) {
  Fp12 r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fp2_mul_fp(a.c1.c0, c_frob2_1());
  r.c0.c1 = fp2_mul_fp(a.c0.c1, c_frob2_2());
  r.c1.c1 = fp2_mul_fp(a.c1.c1, c_frob2_3());
  r.c0.c2 = fp2_mul_fp(a.c0.c2, c_frob2_4());
  r.c1.c2 = fp2_mul_fp(a.c1.c2, c_frob2_5());
  return r;
}

// Granger-Scott squaring for elements of the cyclotomic subgroup G_{Phi_12(p)}.
// View f = g0 + g1 w + g2 w^2 over Fp4 = Fp2[s]/(s^2 - xi), s = w^3, with
// g0 = c0 + c3 s, g1 = c1 + c4 s, g2 = c2 + c5 s (c_k = coefficient of w^k).
//   f^2 = (3 g0^2 - 2 conj(g0)) + (3 s g2^2 + 2 conj(g1)) w + (3 g1^2 - 2 conj(g2)) w^2
// where conj negates the s part.
BLS_HD void fp4_sqr(const Fp2& x, const Fp2& y, Fp2& rx, Fp2& ry) {
  Fp2 t0 = fp2_sqr(x);
  Fp2 t1 = fp2_sqr(y);
  rx = fp2_add(t0, fp2_mul_xi(t1));
  ry = fp2_sub(fp2_sub(fp2_sqr(fp2_add(x, y)), t0), t1);
}

BLS_NOINLINE Fp12 fp12_cyclotomic_sqr(const Fp12& f) {
  // c_k: c0=f.c0.c0 c1=f.c1.c0 c2=f.c0.c1 c3=f.c1.c1 c4=f.c0.c2 c5=f.c1.c2
  Fp2 a0, a1, b0, b1, d0, d1;
  fp4_sqr(f.c0.c0, f.c1.c1, a0, a1);  // g0^2
  fp4_sqr(f.c1.c0, f.c0.c2, b0, b1);  // g1^2
  fp4_sqr(f.c0.c1, f.c1.c2, d0, d1);  // g2^2
  Fp12 r;
  // new g0 = 3 g0^2 - 2 conj(g0):  (3 a0 - 2 c0,  3 a1 + 2 c3)
  r.c0.c0 = fp2_add(fp2_dbl(fp2_sub(a0, f.c0.c0)), a0);
  r.c1.c1 = fp2_add(fp2_dbl(fp2_add(a1, f.c1.c1)), a1);
  // new g1 = 3 s g2^2 + 2 conj(g1):  s (d0 + d1 s) = xi d1 + d0 s
  //   (3 xi d1 + 2 c1,  3 d0 - 2 c4)
  Fp2 xd1 = fp2_mul_xi(d1);
  r.c1.c0 = fp2_add(fp2_dbl(fp2_add(xd1, f.c1.c0)), xd1);
  r.c0.c2 = fp2_add(fp2_dbl(fp2_sub(d0, f.c0.c2)), d0);
  // new g2 = 3 g1^2 - 2 conj(g2):  (3 b0 - 2 c2,  3 b1 + 2 c5)
  r.c0.c1 = fp2_add(fp2_dbl(fp2_sub(b0, f.c0.c1)), b0);
  r.c1.c2 = fp2_add(fp2_dbl(fp2_add(b1, f.c1.c2)), b1);
  return r;
}

}  // namespace bls
