// Cooperative execution: one 64-lane wavefront evaluates one task's Fp circuit.
//
// The tower / pairing formulas are compiled offline (tools/gen_coop.py,
// tools/circuits.py) into level-scheduled steps: in each step every lane performs
// one Fp operation -- a Montgomery product of two short linear combinations of
// frame slots, or a linear combination alone -- reading the task's frame (Fp slots
// in LDS) and the shared constant bank.  An Fp12 product is one step (54 lanes), a
// cyclotomic squaring one product step plus one combination step, the Miller loop
// ~2.3 product steps per bit: the latency of a set's pairing work drops from
// thousands of dependent Fp products in one lane to hundreds of steps.
//
// Step semantics (matched by tools/circuits.py:simulate): all lanes gather their
// operands, the wave synchronises, all lanes write -- so a step may overwrite a
// slot it also reads.  A block is exactly one wavefront, so __syncthreads() is a
// single-wave barrier.
#pragma once

#include "field.hpp"

namespace bls {

#define COOP_LANES 64
#define COOP_FRAME 256
#define COOP_OUT_ZCHECK 0xFFFFu
#define COOP_OUT_NONE 0xFFFEu

struct CoopOp {  // 80 bytes, one per lane per step (tools/gen_coop.py:emit)
  uint16_t out;
  uint8_t kind, na, nb, pad0, pad1, pad2;
  uint16_t a[8];
  uint16_t b[8];
  int16_t ca[8];
  int16_t cb[8];
  uint8_t pad[8];
};

struct CoopProg {
  uint32_t first, n;
};

// Programs of the finalisation frame ("fin", tools/gen_coop.py:build_fin)
struct CoopEnv {
  const CoopOp* ops;
  const Fp* consts;
  CoopProg fin_fmul, fin_g2add, fin_g2dbl, fin_normz, fin_affine, fin_ml_neg_g1, fin_fe1, fin_fe2;
};

// fin frame registers
enum : int {
  FIN_F = 0,
  FIN_G = 12,
  FIN_S = 24,
  FIN_R = 30,
  FIN_Q = 36,
  FIN_INV_IN = 40,
  FIN_INV_OUT = 41,
  FIN_E = 42,
  FIN_HR = 50,
};

// x * c for a small signed integer c (|c| < 2^15)
__device__ __forceinline__ Fp fp_mul_small(const Fp& x, int c) {
  if (c == 1) return x;
  if (c == -1) return fp_neg(x);
  unsigned m = c < 0 ? (unsigned)(-c) : (unsigned)c;
  int top = 31 - __clz(m);
  Fp r = x;
  for (int i = top - 1; i >= 0; --i) {
    r = fp_dbl(r);
    if ((m >> i) & 1u) r = fp_add(r, x);
  }
  return c < 0 ? fp_neg(r) : r;
}

__device__ __forceinline__ Fp lds_load_fp(const Fp* frame, uint32_t slot) {
  const uint4* p = reinterpret_cast<const uint4*>(frame) + 3 * slot;
  uint4 w0 = p[0], w1 = p[1], w2 = p[2];
  Fp r;
  r.l[0] = w0.x; r.l[1] = w0.y; r.l[2] = w0.z; r.l[3] = w0.w;
  r.l[4] = w1.x; r.l[5] = w1.y; r.l[6] = w1.z; r.l[7] = w1.w;
  r.l[8] = w2.x; r.l[9] = w2.y; r.l[10] = w2.z; r.l[11] = w2.w;
  return r;
}

__device__ __forceinline__ void lds_store_fp(Fp* frame, uint32_t slot, const Fp& v) {
  uint4* p = reinterpret_cast<uint4*>(frame) + 3 * slot;
  p[0] = make_uint4(v.l[0], v.l[1], v.l[2], v.l[3]);
  p[1] = make_uint4(v.l[4], v.l[5], v.l[6], v.l[7]);
  p[2] = make_uint4(v.l[8], v.l[9], v.l[10], v.l[11]);
}

__device__ __forceinline__ Fp coop_term(uint16_t ref, const Fp* frame, const Fp* consts) {
  return (ref & 0x8000u) ? consts[ref & 0x7fffu] : lds_load_fp(frame, ref);
}

__device__ __forceinline__ Fp coop_lin(const uint16_t (&refs)[8], const int16_t (&cf)[8], int n,
                                       const Fp* frame, const Fp* consts) {
  Fp acc = fp_zero();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k < n) {
      Fp t = fp_mul_small(coop_term(refs[k], frame, consts), cf[k]);
      acc = k == 0 ? t : fp_add(acc, t);
    }
  }
  return acc;
}

union CoopOpWords {
  uint4 w[5];
  CoopOp op;
};

// Run one program on this block's frame.  *flag (LDS) is set when a zero-check op
// sees zero.
__device__ __noinline__ void coop_run(const CoopEnv& env, CoopProg pg, Fp* frame, uint32_t* flag) {
  const int lane = threadIdx.x;
  const uint4* base = reinterpret_cast<const uint4*>(env.ops);
  for (uint32_t s = 0; s < pg.n; ++s) {
    CoopOpWords u;
    const uint4* src = base + ((size_t)(pg.first + s) * COOP_LANES + lane) * 5;
#pragma unroll
    for (int k = 0; k < 5; ++k) u.w[k] = src[k];
    const CoopOp& op = u.op;
    Fp r = fp_zero();
    if (op.kind != 0) {
      r = coop_lin(op.a, op.ca, op.na, frame, env.consts);
      if (op.kind == 1) r = fp_mul(r, coop_lin(op.b, op.cb, op.nb, frame, env.consts));
    }
    __syncthreads();
    if (op.kind != 0) {
      if (op.out == COOP_OUT_ZCHECK) {
        if (fp_is_zero(r)) *flag = 1u;
      } else {
        lds_store_fp(frame, op.out, r);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Fp inversion by the binary extended Euclidean algorithm (variable time: all
// inputs are public).  ~2 log2(p) shift steps of 12-limb words instead of the
// ~450 dependent Montgomery products of Fermat's a^(p-2).
// In: a in Montgomery form (aR).  Out: a^-1 in Montgomery form (a^-1 R); 0 -> 0.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool big_is_one(const Fp& a) {
  uint32_t acc = a.l[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 12; ++i) acc |= a.l[i];
  return acc == 0;
}

__device__ __forceinline__ void big_shr1(Fp& a) {
#pragma unroll
  for (int i = 0; i < 11; ++i) a.l[i] = (a.l[i] >> 1) | (a.l[i + 1] << 31);
  a.l[11] >>= 1;
}

// a >= b (plain 384-bit)
__device__ __forceinline__ bool big_geq(const Fp& a, const Fp& b) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint64_t t = (uint64_t)a.l[i] - b.l[i] - borrow;
    borrow = (uint32_t)(t >> 63);
  }
  return borrow == 0;
}

__device__ __forceinline__ void big_sub(Fp& a, const Fp& b) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint64_t t = (uint64_t)a.l[i] - b.l[i] - borrow;
    a.l[i] = (uint32_t)t;
    borrow = (uint32_t)(t >> 63);
  }
}

__device__ __noinline__ Fp fp_inv_gcd(Fp a) {
  if (fp_is_zero(a)) return fp_zero();
  Fp u = a, v, x1 = fp_zero(), x2 = fp_zero();
#pragma unroll
  for (int i = 0; i < 12; ++i) v.l[i] = p_limb(i);
  x1.l[0] = 1;
  while (!big_is_one(u) && !big_is_one(v)) {
    while (!(u.l[0] & 1u)) {
      big_shr1(u);
      x1 = fp_half(x1);
    }
    while (!(v.l[0] & 1u)) {
      big_shr1(v);
      x2 = fp_half(x2);
    }
    if (big_geq(u, v)) {
      big_sub(u, v);
      x1 = fp_sub(x1, x2);
    } else {
      big_sub(v, u);
      x2 = fp_sub(x2, x1);
    }
  }
  Fp inv = big_is_one(u) ? x1 : x2;   // (aR)^-1 mod p
  return fp_mul(inv, c_r3());          // (aR)^-1 R^3 / R = a^-1 R
}

// lane 0 inverts frame[in] into frame[out]; the whole block waits
__device__ __forceinline__ void coop_invert(Fp* frame, int in, int out) {
  if (threadIdx.x == 0) lds_store_fp(frame, out, fp_inv_gcd(lds_load_fp(frame, in)));
  __syncthreads();
}

// cooperative copies between global memory and the frame (n slots)
__device__ __forceinline__ void coop_load(Fp* frame, int slot, const Fp* src, int n) {
  for (int k = threadIdx.x; k < n; k += COOP_LANES) lds_store_fp(frame, slot + k, src[k]);
  __syncthreads();
}

__device__ __forceinline__ bool coop_is_zero(const Fp* frame, int slot, int n) {
  bool z = true;
  for (int k = 0; k < n; ++k) z = z && fp_is_zero(lds_load_fp(frame, slot + k));
  return z;
}

}  // namespace bls
