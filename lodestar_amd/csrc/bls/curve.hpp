// BLS12-381 groups G1 (E1/Fp: y^2 = x^3 + 4) and G2 (E2/Fp2: y^2 = x^3 + 4(1+u)).
//
// Jacobian coordinates (x = X/Z^2, y = Y/Z^3; Z = 0 is the point at infinity),
// one point per lane.  The formulas are field-generic (template over Fp / Fp2):
//   dbl-2009-l (2M + 5S), add-2007-bl (11M + 5S), madd-2007-bl (7M + 4S),
// with the exceptional cases (P == Q, P == -Q, infinity) handled explicitly so
// the same code is correct for adversarial signature points that are on the
// curve but outside G2 (subgroup check input).
//
// Replaces blst's p1/p2 arithmetic behind @chainsafe/blst (SURVEY.md 2.2 items
// 2, 3, 5): PublicKey.aggregate (beacon-node/src/chain/bls/utils.ts:11),
// Signature.fromBytes(.., validate=true) (chain/bls/maybeBatch.ts:23,36).
#pragma once

#include "field.hpp"

namespace bls {

// ---- field-generic shims (overloads) ---------------------------------------
BLS_HD Fp f_add(const Fp& a, const Fp& b) { return fp_add(a, b); }
BLS_HD Fp f_sub(const Fp& a, const Fp& b) { return fp_sub(a, b); }
BLS_HD Fp f_mul(const Fp& a, const Fp& b) { return fp_mul(a, b); }
BLS_HD Fp f_sqr(const Fp& a) { return fp_sqr(a); }
BLS_HD Fp f_dbl(const Fp& a) { return fp_dbl(a); }
BLS_HD Fp f_neg(const Fp& a) { return fp_neg(a); }
BLS_HD bool f_is_zero(const Fp& a) { return fp_is_zero(a); }
BLS_HD bool f_eq(const Fp& a, const Fp& b) { return fp_eq(a, b); }
BLS_HD Fp f_inv(const Fp& a) { return fp_inv(a); }
BLS_HD void f_set_zero(Fp& a) { a = fp_zero(); }
BLS_HD void f_set_one(Fp& a) { a = c_one(); }

BLS_HD Fp2 f_add(const Fp2& a, const Fp2& b) { return fp2_add(a, b); }
BLS_HD Fp2 f_sub(const Fp2& a, const Fp2& b) { return fp2_sub(a, b); }
BLS_HD Fp2 f_mul(const Fp2& a, const Fp2& b) { return fp2_mul(a, b); }
BLS_HD Fp2 f_sqr(const Fp2& a) { return fp2_sqr(a); }
BLS_HD Fp2 f_dbl(const Fp2& a) { return fp2_dbl(a); }
BLS_HD Fp2 f_neg(const Fp2& a) { return fp2_neg(a); }
BLS_HD bool f_is_zero(const Fp2& a) { return fp2_is_zero(a); }
BLS_HD bool f_eq(const Fp2& a, const Fp2& b) { return fp2_eq(a, b); }
BLS_HD Fp2 f_inv(const Fp2& a) { return fp2_inv(a); }
BLS_HD void f_set_zero(Fp2& a) { a = fp2_zero(); }
BLS_HD void f_set_one(Fp2& a) { a = fp2_one(); }

template <class F>
struct Jac {
  F x, y, z;
};
template <class F>
struct Aff {
  F x, y;
  bool inf;
};

typedef Jac<Fp> G1J;
typedef Aff<Fp> G1A;
typedef Jac<Fp2> G2J;
typedef Aff<Fp2> G2A;

template <class F>
BLS_HD Jac<F> jac_infinity() {
  Jac<F> r;
  f_set_one(r.x);
  f_set_one(r.y);
  f_set_zero(r.z);
  return r;
}

template <class F>
BLS_HD bool jac_is_inf(const Jac<F>& p) {
  return f_is_zero(p.z);
}

template <class F>
BLS_HD Jac<F> jac_from_aff(const Aff<F>& a) {
  if (a.inf) return jac_infinity<F>();
  Jac<F> r;
  r.x = a.x;
  r.y = a.y;
  f_set_one(r.z);
  return r;
}

template <class F>
BLS_HD Jac<F> jac_neg(const Jac<F>& p) {
  Jac<F> r = p;
  r.y = f_neg(p.y);
  return r;
}

// dbl-2009-l (a = 0).  The order keeps few values live across the out-of-line products
// (each product's callers must hold their live state outside its registers): Z3 first,
// so Y and Z die at once; C8 as soon as C is known.
template <class F>
BLS_HD Jac<F> jac_dbl(const Jac<F>& p) {
  Jac<F> r;
  F B = f_sqr(p.y);
  r.z = f_dbl(f_mul(p.y, p.z));
  F A = f_sqr(p.x);
  F D = f_sqr(f_add(p.x, B));
  F C = f_sqr(B);
  D = f_dbl(f_sub(f_sub(D, A), C));
  const F C8 = f_dbl(f_dbl(f_dbl(C)));
  const F E = f_add(f_dbl(A), A);
  r.x = f_sub(f_sqr(E), f_dbl(D));
  r.y = f_sub(f_mul(E, f_sub(D, r.x)), C8);
  return r;
}

// add-2007-bl with exceptional cases
template <class F>
BLS_HD Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  // ordered so the inputs die early (see jac_dbl): (Z1 + Z2)^2 - Z1Z1 - Z2Z2 right
  // after the Z's last other use
  const F Z1Z1 = f_sqr(p.z);
  const F Z2Z2 = f_sqr(q.z);
  const F S1 = f_mul(f_mul(p.y, q.z), Z2Z2);
  const F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  const F Zs = f_sub(f_sub(f_sqr(f_add(p.z, q.z)), Z1Z1), Z2Z2);
  const F U1 = f_mul(p.x, Z2Z2);
  const F H = f_sub(f_mul(q.x, Z1Z1), U1);
  F rr = f_sub(S2, S1);
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  rr = f_dbl(rr);
  Jac<F> r;
  r.z = f_mul(Zs, H);
  const F I = f_sqr(f_dbl(H));
  const F J = f_mul(H, I);
  const F V = f_mul(U1, I);
  const F S1J2 = f_dbl(f_mul(S1, J));
  r.x = f_sub(f_sub(f_sqr(rr), J), f_dbl(V));
  r.y = f_sub(f_mul(rr, f_sub(V, r.x)), S1J2);
  return r;
}

// madd-2007-bl: p Jacobian + q affine (q not infinity)
template <class F>
BLS_HD Jac<F> jac_add_aff(const Jac<F>& p, const Aff<F>& q) {
  if (q.inf) return p;
  if (jac_is_inf(p)) return jac_from_aff(q);
  const F Z1Z1 = f_sqr(p.z);
  const F H = f_sub(f_mul(q.x, Z1Z1), p.x);
  F rr = f_sub(f_mul(f_mul(q.y, p.z), Z1Z1), p.y);
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  Jac<F> r;
  const F HH = f_sqr(H);
  r.z = f_sub(f_sub(f_sqr(f_add(p.z, H)), Z1Z1), HH);  // Z1 and Z1Z1 die here
  const F I = f_dbl(f_dbl(HH));
  const F J = f_mul(H, I);
  const F YJ2 = f_dbl(f_mul(p.y, J));
  rr = f_dbl(rr);
  const F V = f_mul(p.x, I);
  r.x = f_sub(f_sub(f_sqr(rr), J), f_dbl(V));
  r.y = f_sub(f_mul(rr, f_sub(V, r.x)), YJ2);
  return r;
}

template <class F>
BLS_HD Aff<F> jac_to_aff(const Jac<F>& p) {
  Aff<F> r;
  if (jac_is_inf(p)) {
    f_set_zero(r.x);
    f_set_zero(r.y);
    r.inf = true;
    return r;
  }
  F zi = f_inv(p.z);
  F zi2 = f_sqr(zi);
  r.x = f_mul(p.x, zi2);
  r.y = f_mul(p.y, f_mul(zi2, zi));
  r.inf = false;
  return r;
}

// Jacobian equality (both may be infinity)
template <class F>
BLS_HD bool jac_eq(const Jac<F>& p, const Jac<F>& q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F Z1Z1 = f_sqr(p.z);
  F Z2Z2 = f_sqr(q.z);
  if (!f_eq(f_mul(p.x, Z2Z2), f_mul(q.x, Z1Z1))) return false;
  return f_eq(f_mul(f_mul(p.y, q.z), Z2Z2), f_mul(f_mul(q.y, p.z), Z1Z1));
}

// [k]P for a 64-bit scalar k (left-to-right double-and-add, generic add: safe for
// points of any order).
template <class F>
BLS_HD Jac<F> jac_mul_u64(const Jac<F>& p, uint64_t k) {
  Jac<F> acc = jac_infinity<F>();
  if (k == 0) return acc;
  int top = 63;
  while (!((k >> top) & 1ull)) --top;
  acc = p;
  for (int i = top - 1; i >= 0; --i) {
    acc = jac_dbl(acc);
    if ((k >> i) & 1ull) acc = jac_add(acc, p);
  }
  return acc;
}

// [k]P for an affine base (mixed additions)
template <class F>
BLS_HD Jac<F> aff_mul_u64(const Aff<F>& p, uint64_t k) {
  Jac<F> acc = jac_infinity<F>();
  if (k == 0 || p.inf) return acc;
  int top = 63;
  while (!((k >> top) & 1ull)) --top;
  acc = jac_from_aff(p);
  for (int i = top - 1; i >= 0; --i) {
    acc = jac_dbl(acc);
    if ((k >> i) & 1ull) acc = jac_add_aff(acc, p);
  }
  return acc;
}

// [k]P with a fixed 4-bit window and a caller-provided table T[0..14] = [1..15]P (in
// memory the caller chooses; kernels/k_chain.hip uses the call workspace): 63
// doublings, 13 table additions (mixed when the affine base pa is given) and 15 window
// additions, whatever k -- the form for per-lane scalars, where double-and-add
// executes an addition at every bit for the wavefront.  Complete formulas, so the same
// group element as jac_mul_u64 / aff_mul_u64.
template <class F>
BLS_HD Jac<F> jac_mul_u64_w4(const Jac<F>& p, const Aff<F>* pa, uint64_t k, Jac<F>* T) {
  T[0] = p;  // T[j - 1] = [j] P
  Jac<F> t = jac_dbl(p);
  T[1] = t;
  for (int j = 2; j < 15; ++j) {
    t = pa ? jac_add_aff(t, *pa) : jac_add(t, p);
    T[j] = t;
  }
  const uint32_t top = (uint32_t)(k >> 60);
  Jac<F> acc = top ? T[top - 1] : jac_infinity<F>();
  for (int w = 14; w >= 0; --w) {
    acc = jac_dbl(jac_dbl(jac_dbl(jac_dbl(acc))));
    const uint32_t d = (uint32_t)(k >> (4 * w)) & 15u;
    if (d) acc = jac_add(acc, T[d - 1]);
  }
  return acc;
}

// [k]P for a scalar given as 8 little-endian 32-bit words (secret keys, up to 256 bits)
template <class F>
BLS_HD Jac<F> aff_mul_u256(const Aff<F>& p, const uint32_t k[8]) {
  Jac<F> acc = jac_infinity<F>();
  if (p.inf) return acc;
  for (int i = 255; i >= 0; --i) {
    acc = jac_dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1u) acc = jac_add_aff(acc, p);
  }
  return acc;
}

// [|x|]P, |x| = 0xd201000000010000 (the BLS parameter is x = -|x|)
template <class F>
BLS_HD Jac<F> jac_mul_xabs(const Jac<F>& p) {
  return jac_mul_u64(p, (uint64_t)BLS_X_ABS);
}

// ---- G1 --------------------------------------------------------------------
BLS_HD bool g1_on_curve(const G1A& a) {
  if (a.inf) return true;
  Fp rhs = fp_add(fp_mul(fp_sqr(a.x), a.x), c_b1());
  return fp_eq(fp_sqr(a.y), rhs);
}

BLS_HD G1A g1_generator() {
  G1A g;
  g.x = c_g1_x();
  g.y = c_g1_y();
  g.inf = false;
  return g;
}

// ---- G2 --------------------------------------------------------------------
BLS_HD bool g2_on_curve(const G2A& a) {
  if (a.inf) return true;
  Fp2 rhs = fp2_add(fp2_mul(fp2_sqr(a.x), a.x), c_b2());
  return fp2_eq(fp2_sqr(a.y), rhs);
}

BLS_HD G2A g2_generator() {
  G2A g;
  g.x = c_g2_x();
  g.y = c_g2_y();
  g.inf = false;
  return g;
}

// psi(x, y) = (conj(x) * c_x, conj(y) * c_y) (RFC 9380 Appendix G.3), Jacobian form
BLS_HD G2J g2_psi(const G2J& p) {
  G2J r;
  r.x = fp2_mul(fp2_conj(p.x), c_psi_x());
  r.y = fp2_mul(fp2_conj(p.y), c_psi_y());
  r.z = fp2_conj(p.z);
  return r;
}

// G2 membership: psi(P) == [x]P  (x = -|x|), Scott's test; equals r*P == O on E2.
BLS_HD bool g2_in_subgroup(const G2A& a) {
  if (a.inf) return true;
  G2J p = jac_from_aff(a);
  G2J xp = jac_neg(jac_mul_xabs(p));
  return jac_eq(g2_psi(p), xp);
}

// G1 membership: sigma(P) == [-x^2]P with sigma(x, y) = (beta x, y) (Scott's test,
// "A note on group membership tests for G1, G2 and GT"); equals r*P == O on E1.
BLS_HD bool g1_in_subgroup(const G1A& a) {
  if (a.inf) return true;
  const G1J q = jac_mul_xabs(jac_mul_xabs(jac_from_aff(a)));  // [x^2]P
  if (jac_is_inf(q)) return false;                              // sigma(P) != O
  const Fp z2 = fp_sqr(q.z);
  const Fp z3 = fp_mul(z2, q.z);
  // -[x^2]P == sigma(P):  X == beta x Z^2  and  -Y == y Z^3
  return fp_eq(q.x, fp_mul(fp_mul(c_g1_beta(), a.x), z2)) && fp_eq(fp_neg(q.y), fp_mul(a.y, z3));
}

// Budroni-Pintore cofactor clearing = [h_eff]P (RFC 9380 Appendix G.3)
BLS_HD G2J g2_clear_cofactor(const G2J& p) {
  G2J t1 = jac_neg(jac_mul_xabs(p));  // [x]P
  G2J t2 = g2_psi(p);
  G2J t3 = g2_psi(g2_psi(jac_dbl(p)));
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = jac_neg(jac_mul_xabs(t2));     // [x](t1 + t2)
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(p));
}

// ---- GLV/GLS scalar multiplication by the batch scalar r = a + b mu ----------------
// mu = -x^2 mod r is the eigenvalue of both cheap endomorphisms:
//   G1: sigma(x, y) = (beta x, y) = [-x^2]P                (g1_in_subgroup above)
//   G2: -psi^2(Q) = [-x^2]Q   (psi = [x] on G2, Scott's test above)
// so [a + b mu]P = [a]P + [b]endo(P) with a, b the two 32-bit halves of the set's
// 64-bit random value: 32 doublings instead of 63.  a + b mu is a uniformly drawn
// scalar from 2^64 distinct non-zero values (the lattice {(u, v): u + v mu = 0 mod r}
// has no vector with |u|, |v| < 2^33 but 0, since v x^2 < r for |v| < 2^33), the
// same soundness as blst's 64-bit randomBytesNonZero(8) scalars; the SAME scalar
// multiplies pk in G1 and sig in G2, as the batch equation needs.
BLS_HD G1J g1_sigma(const G1J& p) {
  G1J r = p;
  r.x = fp_mul(p.x, c_g1_beta());  // x = X / Z^2: beta x <-> beta X
  return r;
}

BLS_HD G2J g2_mu(const G2J& p) { return jac_neg(g2_psi(g2_psi(p))); }

// the group's [mu] endomorphism, by point type
BLS_HD G1J jac_endo_mu(const G1J& p) { return g1_sigma(p); }
BLS_HD G2J jac_endo_mu(const G2J& p) { return g2_mu(p); }

// The joint 2-bit-window table T[4 j + i - 1] = [i]P + [j]endo(P), i, j in 0..3, not
// both 0 (15 entries, caller-provided memory) and the 16 windows of (a, b): 33
// doublings and 9 + 1 + 16 additions, whatever a and b (per-lane scalars: the
// wavefront runs every addition anyway).  Complete formulas: the same group element as
// jac_mul on the full scalar.
template <class F>
BLS_HD Jac<F> jac_mul_glv(const Jac<F>& p, uint32_t a, uint32_t b, Jac<F>* T) {
  const Jac<F> p2 = jac_dbl(p);
  const Jac<F> p3 = jac_add(p2, p);
  T[0] = p;
  T[1] = p2;
  T[2] = p3;
  // loops kept rolled: one copy of each formula (the table lives in the caller's memory)
#pragma unroll 1
  for (int j = 1; j < 4; ++j) {
    const Jac<F> e = jac_endo_mu(T[j - 1]);  // [j] endo(P)
    T[4 * j - 1] = e;
#pragma unroll 1
    for (int i = 1; i < 4; ++i) T[4 * j + i - 1] = jac_add(e, T[i - 1]);
  }
  Jac<F> acc = jac_infinity<F>();
#pragma unroll 1
  for (int w = 15; w >= 0; --w) {
    acc = jac_dbl(jac_dbl(acc));
    const uint32_t d = ((a >> (2 * w)) & 3u) | (((b >> (2 * w)) & 3u) << 2);
    if (d) acc = jac_add(acc, T[d - 1]);
  }
  return acc;
}

// the scalar a + b mu mod r as 8 little-endian words (tests / the oracle side)
BLS_HD void glv_split(uint64_t r64, uint32_t& a, uint32_t& b) {
  a = (uint32_t)r64;
  b = (uint32_t)(r64 >> 32);
}

// ---- serialization (ZCash format) ---------------------------------------------
// Error codes follow blst's BLST_ERROR enum; values >= 8 are Lodestar/chainsafe-level.
enum BlsCode : int32_t {
  BLS_OK = 0,
  BLS_BAD_ENCODING = 1,
  BLS_POINT_NOT_ON_CURVE = 2,
  BLS_POINT_NOT_IN_GROUP = 3,
  BLS_PK_IS_INFINITY = 6,
  BLS_INVALID_SIZE = 8,
  BLS_ZERO_SIGNATURE = 9,
  BLS_EMPTY_SET = 10,
  BLS_EMPTY_AGGREGATE = 11,
};

// 96-byte uncompressed G1 (x || y big-endian), blst_p1_deserialize semantics
// (on-curve check, no subgroup check: pubkeys are trusted, pubkeyCache.ts:72-75).
BLS_HD int32_t g1_deserialize96(const uint8_t* b, G1A& out) {
  out.inf = false;
  if (b[0] & 0x80) return BLS_BAD_ENCODING;
  if (b[0] & 0x40) {
    uint8_t acc = b[0] & 0x3f;
    for (int i = 1; i < 96; ++i) acc |= b[i];
    if (acc) return BLS_BAD_ENCODING;
    out.inf = true;
    out.x = fp_zero();
    out.y = fp_zero();
    return BLS_OK;
  }
  if (b[0] & 0x20) return BLS_BAD_ENCODING;
  Fp x = fp_from_be48(b);
  Fp y = fp_from_be48(b + 48);
  if (!fp_plain_is_canonical(x) || !fp_plain_is_canonical(y)) return BLS_BAD_ENCODING;
  out.x = fp_to_mont(x);
  out.y = fp_to_mont(y);
  if (!g1_on_curve(out)) return BLS_POINT_NOT_ON_CURVE;
  return BLS_OK;
}

// 48-byte compressed G1 (pubkey cache load), blst_p1_uncompress semantics.
BLS_HD int32_t g1_decompress48(const uint8_t* b, G1A& out) {
  out.inf = false;
  if (!(b[0] & 0x80)) return BLS_BAD_ENCODING;
  if (b[0] & 0x40) {
    uint8_t acc = b[0] & 0x3f;
    for (int i = 1; i < 48; ++i) acc |= b[i];
    if (acc) return BLS_BAD_ENCODING;
    out.inf = true;
    out.x = fp_zero();
    out.y = fp_zero();
    return BLS_OK;
  }
  uint8_t tmp[48];
  for (int i = 0; i < 48; ++i) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fp x = fp_from_be48(tmp);
  if (!fp_plain_is_canonical(x)) return BLS_BAD_ENCODING;
  out.x = fp_to_mont(x);
  Fp y;
  if (!fp_sqrt(fp_add(fp_mul(fp_sqr(out.x), out.x), c_b1()), y)) return BLS_POINT_NOT_ON_CURVE;
  bool s = (b[0] & 0x20) != 0;
  if (fp_lex_largest(y) != s) y = fp_neg(y);
  out.y = y;
  return BLS_OK;
}

BLS_HD void g1_serialize96(const G1A& a, uint8_t* b) {
  if (a.inf) {
    b[0] = 0x40;
    for (int i = 1; i < 96; ++i) b[i] = 0;
    return;
  }
  fp_to_be48(fp_from_mont(a.x), b);
  fp_to_be48(fp_from_mont(a.y), b + 48);
}

BLS_HD void g1_compress48(const G1A& a, uint8_t* b) {
  if (a.inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 48; ++i) b[i] = 0;
    return;
  }
  fp_to_be48(fp_from_mont(a.x), b);
  b[0] |= 0x80;
  if (fp_lex_largest(a.y)) b[0] |= 0x20;
}

// 96-byte compressed G2 signature, blst_p2_uncompress semantics (no subgroup check)
BLS_HD int32_t g2_decompress96(const uint8_t* b, G2A& out) {
  out.inf = false;
  if (!(b[0] & 0x80)) return BLS_BAD_ENCODING;
  if (b[0] & 0x40) {
    uint8_t acc = b[0] & 0x3f;
    for (int i = 1; i < 96; ++i) acc |= b[i];
    if (acc) return BLS_BAD_ENCODING;
    out.inf = true;
    out.x = fp2_zero();
    out.y = fp2_zero();
    return BLS_OK;
  }
  uint8_t tmp[48];
  for (int i = 0; i < 48; ++i) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fp x1 = fp_from_be48(tmp);
  Fp x0 = fp_from_be48(b + 48);
  if (!fp_plain_is_canonical(x1) || !fp_plain_is_canonical(x0)) return BLS_BAD_ENCODING;
  out.x = Fp2{fp_to_mont(x0), fp_to_mont(x1)};
  Fp2 y;
  if (!fp2_sqrt(fp2_add(fp2_mul(fp2_sqr(out.x), out.x), c_b2()), y)) return BLS_POINT_NOT_ON_CURVE;
  bool s = (b[0] & 0x20) != 0;
  if (fp2_lex_largest(y) != s) y = fp2_neg(y);
  out.y = y;
  return BLS_OK;
}

// 192-byte uncompressed G2: x.c1 || x.c0 || y.c1 || y.c0
BLS_HD void g2_serialize192(const G2A& a, uint8_t* b) {
  if (a.inf) {
    b[0] = 0x40;
    for (int i = 1; i < 192; ++i) b[i] = 0;
    return;
  }
  fp_to_be48(fp_from_mont(a.x.c1), b);
  fp_to_be48(fp_from_mont(a.x.c0), b + 48);
  fp_to_be48(fp_from_mont(a.y.c1), b + 96);
  fp_to_be48(fp_from_mont(a.y.c0), b + 144);
}

BLS_HD void g2_compress96(const G2A& a, uint8_t* b) {
  if (a.inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 96; ++i) b[i] = 0;
    return;
  }
  fp_to_be48(fp_from_mont(a.x.c1), b);
  fp_to_be48(fp_from_mont(a.x.c0), b + 48);
  b[0] |= 0x80;
  if (fp2_lex_largest(a.y)) b[0] |= 0x20;
}

}  // namespace bls
