// Fp6 / Fp12 over the lazy 28-bit-digit coefficients of lazy28.hpp, for the f side of the
// Miller loops (kernels/k_mlq.hip k_mlf): the same formulas as field.hpp's fp6_mul /
// fp6_mul_01 / fp6_mul_1 / fp12_sqr / fp12_mul_line / fp12_mul_line2, with every
// addition and subtraction a digit-wise one and the bounds carried in the types (an
// operand is normalised only where a product's columns or a digit would overflow, decided
// at compile time).  An Fp6 / Fp12 keeps one coefficient type (the widest of its parts).
// Test: tests/test_lazy28.py::test_lazy28_fp12_ops (bit-exact against field.hpp).
#pragma once

#include "lazy28.hpp"

namespace bls {

template <class T>
struct L6 {
  L2<T> c0, c1, c2;
};
template <class T>
struct L12 {
  L6<T> c0, c1;
};

template <class A, class B, class C>
BLS_HD auto l6_make(const L2<A>& a, const L2<B>& b, const L2<C>& c) {
  typedef LzMax<LzMax<A, B>, C> T;
  return L6<T>{l2_widen<T>(a), l2_widen<T>(b), l2_widen<T>(c)};
}
template <class To, class A>
BLS_HD L6<To> l6_widen(const L6<A>& a) {
  return L6<To>{l2_widen<To>(a.c0), l2_widen<To>(a.c1), l2_widen<To>(a.c2)};
}
template <class A, class B>
BLS_HD auto l6_add(const L6<A>& a, const L6<B>& b) {
  return l6_make(l2_add(a.c0, b.c0), l2_add(a.c1, b.c1), l2_add(a.c2, b.c2));
}
template <class A, class B>
BLS_HD auto l6_sub(const L6<A>& a, const L6<B>& b) {
  return l6_make(l2_sub(a.c0, b.c0), l2_sub(a.c1, b.c1), l2_sub(a.c2, b.c2));
}
template <class A>
BLS_HD L6<A> l6_neg(const L6<A>& a) {
  return L6<A>{l2_neg(a.c0), l2_neg(a.c1), l2_neg(a.c2)};
}
template <class A>
BLS_HD auto l6_norm(const L6<A>& a) {
  return l6_make(l2_norm(a.c0), l2_norm(a.c1), l2_norm(a.c2));
}
// a v = (xi a2, a0, a1)
template <class A>
BLS_HD auto l6_mul_v(const L6<A>& a) {
  return l6_make(l2_mul_xi(a.c2), a.c0, a.c1);
}
// Karatsuba over Fp2: 6 Fp2 products (field.hpp fp6_mul)
template <class A, class B>
BLS_HD auto l6_mul(const L6<A>& a, const L6<B>& b) {
  const auto t0 = l2_mul(a.c0, b.c0);
  const auto t1 = l2_mul(a.c1, b.c1);
  const auto t2 = l2_mul(a.c2, b.c2);
  const auto c0 = l2_add(l2_mul_xi(l2_sub(l2_sub(l2_mul(l2_add(a.c1, a.c2), l2_add(b.c1, b.c2)), t1), t2)), t0);
  const auto c1 = l2_add(l2_sub(l2_sub(l2_mul(l2_add(a.c0, a.c1), l2_add(b.c0, b.c1)), t0), t1), l2_mul_xi(t2));
  const auto c2 = l2_add(l2_sub(l2_sub(l2_mul(l2_add(a.c0, a.c2), l2_add(b.c0, b.c2)), t0), t2), t1);
  return l6_make(c0, c1, c2);
}
// a (d0 + d1 v): 5 Fp2 products (field.hpp fp6_mul_01)
template <class A, class B, class C>
BLS_HD auto l6_mul_01(const L6<A>& a, const L2<B>& d0, const L2<C>& d1) {
  const auto a0d0 = l2_mul(a.c0, d0);
  const auto a1d1 = l2_mul(a.c1, d1);
  const auto c0 = l2_add(a0d0, l2_mul_xi(l2_mul(a.c2, d1)));
  const auto c1 = l2_sub(l2_sub(l2_mul(l2_add(a.c0, a.c1), l2_add(d0, d1)), a0d0), a1d1);
  const auto c2 = l2_add(a1d1, l2_mul(a.c2, d0));
  return l6_make(c0, c1, c2);
}
// a (d1 v): 3 Fp2 products (field.hpp fp6_mul_1)
template <class A, class B>
BLS_HD auto l6_mul_1(const L6<A>& a, const L2<B>& d1) {
  return l6_make(l2_mul_xi(l2_mul(a.c2, d1)), l2_mul(a.c0, d1), l2_mul(a.c1, d1));
}

template <class A, class B>
BLS_HD auto l12_make(const L6<A>& a, const L6<B>& b) {
  typedef LzMax<A, B> T;
  return L12<T>{l6_widen<T>(a), l6_widen<T>(b)};
}
template <class To, class A>
BLS_HD L12<To> l12_widen(const L12<A>& a) {
  return L12<To>{l6_widen<To>(a.c0), l6_widen<To>(a.c1)};
}
template <class A>
BLS_HD L12<A> l12_conj(const L12<A>& a) {
  return L12<A>{a.c0, l6_neg(a.c1)};
}
template <class A>
BLS_HD auto l12_norm(const L12<A>& a) {
  return l12_make(l6_norm(a.c0), l6_norm(a.c1));
}
template <class A>
BLS_HD L6<LzN<2>> l6_reduce(const L6<A>& a) {
  return L6<LzN<2>>{l2_reduce(a.c0), l2_reduce(a.c1), l2_reduce(a.c2)};
}
// every coefficient back to |value| < 2 p (lz_reduce): the Miller loop's f between steps
template <class A>
BLS_HD L12<LzN<2>> l12_reduce(const L12<A>& a) {
  return L12<LzN<2>>{l6_reduce(a.c0), l6_reduce(a.c1)};
}

// complex squaring (field.hpp fp12_sqr): (A + B w)^2 = (s - ab - v ab) + 2 ab w,
// ab = A B, s = (A + B)(A + v B)
template <class A>
BLS_HD auto l12_sqr(const L12<A>& a) {
  const auto ab = l6_mul(a.c0, a.c1);
  const auto s = l6_mul(l6_add(a.c0, a.c1), l6_add(a.c0, l6_mul_v(a.c1)));
  return l12_make(l6_sub(l6_sub(s, ab), l6_mul_v(ab)), l6_add(ab, ab));
}
// f (l0 + l2 w^2 + l3 w^3) (field.hpp fp12_mul_line)
template <class F, class L>
BLS_HD auto l12_mul_line(const L12<F>& f, const L2<L>& l0, const L2<L>& l2, const L2<L>& l3) {
  const auto aa = l6_mul_01(f.c0, l0, l2);
  const auto bb = l6_mul_1(f.c1, l3);
  const auto c1 = l6_sub(l6_sub(l6_mul_01(l6_add(f.c0, f.c1), l0, l2_add(l2, l3)), aa), bb);
  return l12_make(l6_add(aa, l6_mul_v(bb)), c1);
}
// f L M for two lines (field.hpp fp12_mul_line2): the lines' product first (6 Fp2
// products), then f P by Karatsuba over Fp6 (6 + 5 + 6): 23 Fp2 products
template <class F, class L>
BLS_HD auto l12_mul_line2(const L12<F>& f, const L2<L>& l0, const L2<L>& l2, const L2<L>& l3, const L2<L>& m0,
                          const L2<L>& m2, const L2<L>& m3) {
  const auto m00 = l2_mul(l0, m0), m22 = l2_mul(l2, m2), m33 = l2_mul(l3, m3);
  const auto a0 = l2_add(m00, l2_mul_xi(m33));
  const auto a2 = l2_sub(l2_sub(l2_mul(l2_add(l0, l2), l2_add(m0, m2)), m00), m22);
  const auto a3 = l2_sub(l2_sub(l2_mul(l2_add(l0, l3), l2_add(m0, m3)), m00), m33);
  const auto a5 = l2_sub(l2_sub(l2_mul(l2_add(l2, l3), l2_add(m2, m3)), m22), m33);
  const auto p0 = l6_make(a0, a2, m22);
  const auto t0 = l6_mul(f.c0, p0);
  const auto t1 = l6_mul_v(l6_mul_01(f.c1, a3, a5));  // f.c1 (a3 v + a5 v^2)
  const auto c1 = l6_sub(l6_sub(l6_mul(l6_add(f.c0, f.c1), l6_make(a0, l2_add(a2, a3), l2_add(m22, a5))), t0), t1);
  return l12_make(l6_add(t0, l6_mul_v(t1)), c1);
}

// ---- the line side (kernels/k_mlq.hip k_mlq) ------------------------------------------
// pairing.hpp's miller_dbl_step / miller_add_step in the lazy form, each followed by the
// line's evaluation at the prepared G1 point (l0 z^3, l2 XZ, l3 Y: products, so the three
// line coefficients come out normalised with |value| < 2 p, the form k_mlf reads).
// T = LzN<2>: every coordinate a product's output or reduced (lz_reduce), so the type closes
template <class T>
struct LProj {
  L2<T> x, y, z;
};
typedef LzN<2> LzL;  // a stored line coefficient
template <class P>
struct LEval {
  P xz, y, z3;
};

template <class T, class P>
BLS_HD void lz_dbl_line(LProj<T>& t, const LEval<P>& e1, L2<LzL> l[3]) {
  const auto a = l2_half(l2_mul(t.x, t.y));
  const auto b = l2_sqr(t.y);
  const auto c = l2_sqr(t.z);
  const auto e = l2_mul_xi(l2_mulc<4>(l2_norm(l2_mulc<3>(c))));  // 3 b' c, b' = 4 (1 + u)
  const auto f = l2_mulc<3>(e);
  const auto g = l2_half(l2_add(b, f));
  const auto h = l2_sub(l2_sqr(l2_add(t.y, t.z)), l2_add(b, c));
  const auto i = l2_sub(e, b);
  const auto j = l2_sqr(t.x);
  const auto e2 = l2_sqr(e);
  t.x = l2_widen<T>(l2_mul(a, l2_sub(b, f)));
  t.y = l2_widen<T>(l2_reduce(l2_sub(l2_sqr(g), l2_mulc<3>(e2))));  // the one sum T keeps
  t.z = l2_widen<T>(l2_mul(b, h));
  l[0] = l2_widen<LzL>(l2_mul_fp(i, e1.z3));
  l[1] = l2_widen<LzL>(l2_mul_fp(l2_mulc<3>(j), e1.xz));
  l[2] = l2_widen<LzL>(l2_mul_fp(l2_neg(h), e1.y));
}

template <class T, class Q, class P>
BLS_HD void lz_add_line(LProj<T>& t, const L2<Q>& qx, const L2<Q>& qy, const LEval<P>& e1, L2<LzL> l[3]) {
  const auto theta = l2_sub(t.y, l2_mul(qy, t.z));
  const auto lambda = l2_sub(t.x, l2_mul(qx, t.z));
  const auto c = l2_sqr(theta);
  const auto d = l2_sqr(lambda);
  const auto e = l2_mul(lambda, d);
  const auto f = l2_mul(t.z, c);
  const auto g = l2_mul(t.x, d);
  const auto h = l2_sub(l2_add(e, f), l2_dbl(g));
  const auto ty = l2_sub(l2_mul(theta, l2_sub(g, h)), l2_mul(e, t.y));
  t.x = l2_widen<T>(l2_mul(lambda, h));
  t.y = l2_widen<T>(l2_reduce(ty));
  t.z = l2_widen<T>(l2_mul(t.z, e));
  l[0] = l2_widen<LzL>(l2_mul_fp(l2_sub(l2_mul(theta, qx), l2_mul(lambda, qy)), e1.z3));
  l[1] = l2_widen<LzL>(l2_mul_fp(l2_neg(theta), e1.xz));
  l[2] = l2_widen<LzL>(l2_mul_fp(lambda, e1.y));
}

}  // namespace bls
