// hash_to_G2 for the POP ciphersuite (RFC 9380 suite BLS12381G2_XMD:SHA-256_SSWU_RO_,
// DST "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"), one message per lane.
//
// The reference reaches this through blst's Pairing.mul_n_aggregate / verify
// ([ext] @chainsafe/blst).  Messages on the hot
// path are 32-byte signing roots (state-transition/src/util/signingRoot.ts:7-13),
// so expand_message_xmd is specialised to len(msg) = 32, len_in_bytes = 256:
// 18 SHA-256 compressions, the all-zero Z_pad block folded into a precomputed
// midstate and every DST-dependent word a compile-time constant.
#pragma once

#include "curve.hpp"

namespace bls {

BLS_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

BLS_HD uint32_t sha256_k(int i) {
  const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  return K[i];
}

// One SHA-256 compression of the 16 big-endian words W into state s.
BLS_NOINLINE void sha256_compress(uint32_t s[8], const uint32_t Win[16]) {
  uint32_t W[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) W[i] = Win[i];
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = W[i];
    } else {
      uint32_t w15 = W[(i + 1) & 15], w2 = W[(i + 14) & 15];
      uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = W[i & 15] + s0 + W[(i + 9) & 15] + s1;
      W[i & 15] = wi;
    }
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + sha256_k(i) + wi;
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  s[0] += a;
  s[1] += b;
  s[2] += c;
  s[3] += d;
  s[4] += e;
  s[5] += f;
  s[6] += g;
  s[7] += h;
}

BLS_HD void sha256_init(uint32_t s[8]) {
  s[0] = 0x6a09e667u;
  s[1] = 0xbb67ae85u;
  s[2] = 0x3c6ef372u;
  s[3] = 0xa54ff53au;
  s[4] = 0x510e527fu;
  s[5] = 0x9b05688cu;
  s[6] = 0x1f83d9abu;
  s[7] = 0x5be0cd19u;
}

// expand_message_xmd(msg, DST, 256) for a 32-byte message given as 8 big-endian
// words; output 64 big-endian words (uniform_bytes).
BLS_HD void expand_message_xmd_32(const uint32_t msg[8], uint32_t out[64]) {
  uint32_t W[16];
  uint32_t b0[8];
  // b0 = H(Z_pad || msg || I2OSP(256, 2) || I2OSP(0, 1) || DST')
#pragma unroll
  for (int i = 0; i < 8; ++i) b0[i] = sha_zpad_mid(i);
#pragma unroll
  for (int i = 0; i < 8; ++i) W[i] = msg[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) W[8 + i] = xmd_b0_blk2_tail(i);
  sha256_compress(b0, W);
#pragma unroll
  for (int i = 0; i < 16; ++i) W[i] = xmd_b0_blk3(i);
  sha256_compress(b0, W);
  // b_i = H(strxor(b0, b_{i-1}) || I2OSP(i, 1) || DST'), b_0' = zeros
  uint32_t prev[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) prev[i] = 0;
  for (int blk = 1; blk <= 8; ++blk) {
    uint32_t s[8];
    sha256_init(s);
#pragma unroll
    for (int i = 0; i < 8; ++i) W[i] = b0[i] ^ prev[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) W[8 + i] = xmd_bi_blkA_tail(i);
    W[8] |= (uint32_t)blk << 24;
    sha256_compress(s, W);
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = xmd_bi_blkB(i);
    sha256_compress(s, W);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      prev[i] = s[i];
      out[(blk - 1) * 8 + i] = s[i];
    }
  }
}

// 64 big-endian bytes (16 words, most significant first) -> Montgomery Fp of the
// value mod p:  v = hi * 2^256 + lo with hi, lo < 2^256 < p.
BLS_HD Fp fp_from_be64_words(const uint32_t w[16]) {
  Fp hi = fp_zero(), lo = fp_zero();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    hi.l[k] = w[7 - k];
    lo.l[k] = w[15 - k];
  }
  return fp_add(fp_mul(hi, c_2e256_r2()), fp_mul(lo, c_r2()));
}

BLS_HD void hash_to_field_fp2_x2(const uint32_t msg[8], Fp2& u0, Fp2& u1) {
  uint32_t ub[64];
  expand_message_xmd_32(msg, ub);
  u0.c0 = fp_from_be64_words(ub + 0);
  u0.c1 = fp_from_be64_words(ub + 16);
  u1.c0 = fp_from_be64_words(ub + 32);
  u1.c1 = fp_from_be64_words(ub + 48);
}

// Simplified SWU onto E2': y^2 = x^3 + A'x + B' (RFC 9380 6.6.2)
BLS_HD G2A map_to_curve_sswu(const Fp2& u) {
  const Fp2 A = c_sswu_a(), B = c_sswu_b(), Z = c_sswu_z();
  Fp2 u2 = fp2_sqr(u);
  Fp2 zu2 = fp2_mul(Z, u2);
  Fp2 den = fp2_add(fp2_sqr(zu2), zu2);
  Fp2 x1;
  if (fp2_is_zero(den)) {
    x1 = c_sswu_b_over_za();
  } else {
    x1 = fp2_mul(c_sswu_mb_over_a(), fp2_add(fp2_one(), fp2_inv(den)));
  }
  Fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), A), x1), B);
  G2A r;
  r.inf = false;
  Fp2 y;
  if (fp2_sqrt(gx1, y)) {
    r.x = x1;
  } else {
    r.x = fp2_mul(zu2, x1);
    Fp2 gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(r.x), A), r.x), B);
    fp2_sqrt(gx2, y);  // gx2 = Z^3 u^6 gx1 is a square when gx1 is not
  }
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  r.y = y;
  return r;
}

// Simplified SWU with two Fp exponentiations whichever branch is taken (the
// verify pipeline's stage_pre_sswu).  Same output as map_to_curve_sswu:
//   * 1/den by one Fp inversion of the norm (binary GCD);
//   * g(x1) is a square in Fp2 iff N(g(x1)) is a square in Fp, decided by
//     gamma = N(g(x1))^((p+1)/4): gamma^2 == N  ->  x = x1, sqrt(N) = gamma;
//     otherwise gamma^2 == -N and, g(x2) = Z^3 u^6 g(x1) with N(Z) = 5,
//     sqrt(N(g(x2))) = N(u)^3 sqrt(-125) gamma  (no second Legendre exponentiation);
//   * the Fp2 root from sqrt(N) as in fp2_sqrt (one (p-3)/4 exponentiation); the
//     sign of sqrt(N) does not matter since y is normalised by sgn0(u).
// Returns false (the caller falls back to the exact routine) when den == 0, when
// g(x).c1 == 0 (fp2_sqrt's special case) or if the root does not verify.
BLS_HD bool map_to_curve_sswu_fast(const Fp2& u, Fp2& xo, Fp2& yo) {
  const Fp2 A = c_sswu_a(), B = c_sswu_b(), Z = c_sswu_z();
  Fp2 u2 = fp2_sqr(u);
  Fp2 zu2 = fp2_mul(Z, u2);
  Fp2 den = fp2_add(fp2_sqr(zu2), zu2);
  if (fp2_is_zero(den)) return false;
  Fp nd = fp_add(fp_sqr(den.c0), fp_sqr(den.c1));
  Fp ndi = fp_inv_gcd(nd);
  Fp2 deninv = Fp2{fp_mul(den.c0, ndi), fp_neg(fp_mul(den.c1, ndi))};
  Fp2 x = fp2_mul(c_sswu_mb_over_a(), fp2_add(fp2_one(), deninv));
  Fp2 gx = fp2_add(fp2_mul(fp2_add(fp2_sqr(x), A), x), B);
  Fp n1 = fp_add(fp_sqr(gx.c0), fp_sqr(gx.c1));
  Fp gamma = fp_pow_const<e_p_plus_1_div_4, E_P_PLUS_1_DIV_4_BITS>(n1);
  if (!fp_eq(fp_sqr(gamma), n1)) {
    x = fp2_mul(zu2, x);
    gx = fp2_add(fp2_mul(fp2_add(fp2_sqr(x), A), x), B);
    Fp nu = fp_add(fp_sqr(u.c0), fp_sqr(u.c1));
    gamma = fp_mul(fp_mul(fp_mul(fp_sqr(nu), nu), c_sqrt_m125()), gamma);
  }
  if (fp_is_zero(gx.c1)) return false;
  Fp d = fp_half(fp_add(gx.c0, gamma));
  Fp t = fp_pow_const<e_p_minus_3_div_4, E_P_MINUS_3_DIV_4_BITS>(d);
  Fp dt = fp_mul(d, t);
  Fp a1t2 = fp_half(fp_mul(gx.c1, t));
  Fp2 y = fp_eq(fp_sqr(dt), d) ? Fp2{dt, a1t2} : Fp2{a1t2, fp_neg(dt)};
  if (!fp2_eq(fp2_sqr(y), gx)) return false;
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  xo = x;
  yo = y;
  return true;
}

// 3-isogeny E2' -> E2 (RFC 9380 Appendix E.3), affine
BLS_HD G2A iso_map_g2(const G2A& p) {
  const Fp2 x = p.x;
  Fp2 xn = c_iso_xnum_3();
  xn = fp2_add(fp2_mul(xn, x), c_iso_xnum_2());
  xn = fp2_add(fp2_mul(xn, x), c_iso_xnum_1());
  xn = fp2_add(fp2_mul(xn, x), c_iso_xnum_0());
  Fp2 xd = fp2_add(x, c_iso_xden_1());  // monic, degree 2
  xd = fp2_add(fp2_mul(xd, x), c_iso_xden_0());
  Fp2 yn = c_iso_ynum_3();
  yn = fp2_add(fp2_mul(yn, x), c_iso_ynum_2());
  yn = fp2_add(fp2_mul(yn, x), c_iso_ynum_1());
  yn = fp2_add(fp2_mul(yn, x), c_iso_ynum_0());
  Fp2 yd = fp2_add(x, c_iso_yden_2());  // monic, degree 3
  yd = fp2_add(fp2_mul(yd, x), c_iso_yden_1());
  yd = fp2_add(fp2_mul(yd, x), c_iso_yden_0());
  G2A r;
  if (p.inf || fp2_is_zero(xd) || fp2_is_zero(yd)) {
    r.inf = true;
    r.x = fp2_zero();
    r.y = fp2_zero();
    return r;
  }
  // one inversion for both denominators
  Fp2 inv = fp2_inv(fp2_mul(xd, yd));
  r.x = fp2_mul(xn, fp2_mul(inv, yd));
  r.y = fp2_mul(fp2_mul(p.y, yn), fp2_mul(inv, xd));
  r.inf = false;
  return r;
}

// 3-isogeny E2' -> E2 (RFC 9380 Appendix E.3) into Jacobian coordinates:
// x = xn / xd, y = y' yn / yd  ->  Z = xd yd, X = xn xd yd^2, Y = y' yn xd^3 yd^2.
// A zero denominator gives Z = 0, the point at infinity (iso_map_g2's convention).
BLS_HD G2J iso_map_jac(const Fp2& x, const Fp2& y) {
  Fp2 xn = c_iso_xnum_3();
  xn = fp2_add(fp2_mul(xn, x), c_iso_xnum_2());
  xn = fp2_add(fp2_mul(xn, x), c_iso_xnum_1());
  xn = fp2_add(fp2_mul(xn, x), c_iso_xnum_0());
  Fp2 xd = fp2_add(x, c_iso_xden_1());
  xd = fp2_add(fp2_mul(xd, x), c_iso_xden_0());
  Fp2 yn = c_iso_ynum_3();
  yn = fp2_add(fp2_mul(yn, x), c_iso_ynum_2());
  yn = fp2_add(fp2_mul(yn, x), c_iso_ynum_1());
  yn = fp2_add(fp2_mul(yn, x), c_iso_ynum_0());
  Fp2 yd = fp2_add(x, c_iso_yden_2());
  yd = fp2_add(fp2_mul(yd, x), c_iso_yden_1());
  yd = fp2_add(fp2_mul(yd, x), c_iso_yden_0());
  const Fp2 yd2 = fp2_sqr(yd);
  const Fp2 xd2 = fp2_sqr(xd);
  G2J r;
  r.z = fp2_mul(xd, yd);
  r.x = fp2_mul(fp2_mul(xn, xd), yd2);
  r.y = fp2_mul(fp2_mul(fp2_mul(y, yn), fp2_mul(xd2, xd)), yd2);
  if (fp2_is_zero(r.z)) return jac_infinity<Fp2>();
  return r;
}

// hash_to_G2 of a 32-byte message (8 big-endian words), Jacobian output
BLS_HD G2J hash_to_g2_jac(const uint32_t msg[8]) {
  Fp2 u0, u1;
  hash_to_field_fp2_x2(msg, u0, u1);
  G2A q0 = iso_map_g2(map_to_curve_sswu(u0));
  G2A q1 = iso_map_g2(map_to_curve_sswu(u1));
  G2J s = jac_add_aff(jac_from_aff(q0), q1);
  return g2_clear_cofactor(s);
}

BLS_HD G2A hash_to_g2(const uint32_t msg[8]) { return jac_to_aff(hash_to_g2_jac(msg)); }

BLS_HD void msg_words_from_bytes(const uint8_t* m, uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    w[i] = ((uint32_t)m[4 * i] << 24) | ((uint32_t)m[4 * i + 1] << 16) | ((uint32_t)m[4 * i + 2] << 8) |
           (uint32_t)m[4 * i + 3];
}

}  // namespace bls
