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
#define COOP_OUT_NONE 0xFFFEu   // lane idle (kind 0, never written)
#define COOP_OUT_ZSET 0xFFF0u   // zero-check of packed set s >= 1: 0xFFF0 + s
#define COOP_MAX_CONSTS 40  // constants staged per block (tools/gen_coop.py asserts the bank fits)
// op kinds (tools/gen_coop.py emit, lane_entries): 0 idle, 1 product of two combinations,
// 2 combination (or its part in a lane group), 3 / 4 part of a product's operand a / b in
// a lane group
#define COOP_MUL 1u
#define COOP_LIN 2u
#define COOP_GRP_A 3u
#define COOP_GRP_B 4u

struct CoopOp {  // 80 bytes, one per lane per step (tools/gen_coop.py:emit)
  uint16_t out;
  uint8_t kind, na, nb;
  uint8_t ma, mb, flags;  // the same on every lane of a step: largest na over the lanes that
                          // gather a, largest nb over the ungrouped products; bit 0 / 1: a / b
                          // is one +1 term on every one of them; bits 2-3 / 4-5: log2 of the
                          // lane-group size of the step's products / combinations
  uint16_t a[8];
  uint16_t b[8];
  int16_t ca[8];
  int16_t cb[8];
  uint8_t pad[8];
};

struct CoopProg {
  uint32_t first, n;
};

// Per-block LDS of a cooperative task: the frame, then the constant bank, so one
// slot index (constants at COOP_FRAME + k, tools/gen_coop.py:emit) addresses both.
struct CoopLds {
  Fp frame[COOP_FRAME];
  Fp cbank[COOP_MAX_CONSTS];
  uint32_t flag;
};
static_assert(offsetof(CoopLds, cbank) == COOP_FRAME * sizeof(Fp), "constant bank must follow the frame");

// LDS of a task whose programs were scheduled for a FRAME_N-slot frame (constants at
// slot FRAME_N + k, tools/gen_coop.py:emit)
template <int FRAME_N>
struct CoopLdsN {
  Fp frame[FRAME_N];
  Fp cbank[COOP_MAX_CONSTS];
  uint32_t flag;
};

#define COOP_FRAME2 380  // the 2-set packed programs (tools/gen_coop.py FRAME2): with the
                         // 40-constant bank 20.2 KB of LDS, 8 blocks = 2 wavefronts per SIMD
#define COOP_FRAME3 640  // the 3-set packed programs (tools/gen_coop.py FRAME3)

// Programs of S sets packed in one wavefront (tools/gen_pset.py build_pset(S)):
// add[(xb << S) | rmask], bit s of rmask = r bit of packed set s; add[0] unused
struct CoopPsetN {
  CoopProg prep, dbl_all, add_x, phase2, norm2, affine2, ml2;
};

// Programs of the finalisation frame ("fin", tools/gen_coop.py:build_fin)
struct CoopEnv {
  const CoopOp* ops;
  const Fp* consts;
  uint32_t n_consts;
  CoopProg fin_fmul, fin_fe1, fin_fe2;
  CoopProg fin_fe2_w2;  // fin_fe2 laid out for two wavefronts (k_indiv_coop2)
  // per-set frame (tools/gen_pset.py, kernels/k_pset.hip; the r chains run beside them)
  CoopProg pset_prep, pset_dbl_all, pset_add_x, pset_phase2, pset_norm2, pset_affine2, pset_ml2;
  CoopProg pset_ml2_w2;  // pset_ml2 laid out for two wavefronts (k_pset: every product on a lane pair)
  CoopProg pset_xchain;  // the |x| chains as one program (pset_dbl_all / pset_add_x by the bits of |x|)
  CoopPsetN packed[2];  // [0]: 2 sets per wavefront, [1]: 3 sets
  // single-pair Miller loops (tools/gen_pset.py build_ml1, kernels/k_pset.hip k_mln, the
  // cooperative packings tests force): 1 or 2 sets per wavefront (COOP_FRAME)
  CoopProg ml1_1, ml1_2;
  // the device copy of this struct (bls_gpu.hip load_coop_tables): kernels take it by
  // pointer -- by value it made their arguments (with PipeBufs) ~830 bytes
  const CoopEnv* dev;
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

// The same through an explicit LDS (address space 3) pointer: 32-bit addressing with
// no generic-pointer checks per access (the interpreter converts its frame once).
typedef unsigned int bls_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int bls_u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) bls_u32x4 LdsU4;

__device__ __forceinline__ Fp lds_load_fp(const LdsU4* base, uint32_t slot) {
  const LdsU4* p = base + 3 * slot;
  bls_u32x4 w0 = p[0], w1 = p[1], w2 = p[2];
  Fp r;
  r.l[0] = w0.x; r.l[1] = w0.y; r.l[2] = w0.z; r.l[3] = w0.w;
  r.l[4] = w1.x; r.l[5] = w1.y; r.l[6] = w1.z; r.l[7] = w1.w;
  r.l[8] = w2.x; r.l[9] = w2.y; r.l[10] = w2.z; r.l[11] = w2.w;
  return r;
}

__device__ __forceinline__ void lds_store_fp(LdsU4* base, uint32_t slot, const Fp& v) {
  LdsU4* p = base + 3 * slot;
  p[0] = bls_u32x4{v.l[0], v.l[1], v.l[2], v.l[3]};
  p[1] = bls_u32x4{v.l[4], v.l[5], v.l[6], v.l[7]};
  p[2] = bls_u32x4{v.l[8], v.l[9], v.l[10], v.l[11]};
}

// Lazy linear combination: terms accumulate unreduced in a 13-limb two's-complement
// accumulator (|sum| < 8 * 2^15 * p < 2^399); one reduction at the end.
struct Acc13 {
  uint32_t l[13];
};

__device__ __forceinline__ uint32_t k20p_limb(int i) {  // 2^20 * p, 13 limbs
  const uint32_t t[13] = {0xaab00000u, 0xfffffffau, 0xfffb9fefu, 0xffeb153fu, 0x6241eabfu, 0x2a0f6b0fu, 0x2bf6730du,
                          0xb84f3851u, 0xcd764774u, 0x7b6434bau, 0x69a4b1bau, 0x1ea397feu, 0x0001a011u};
  return t[i];
}

// (sum + extra) mod p of the accumulator as a value in [0, 3p) (the interpreter's
// lazy representation); extra < 2^20 (the |c| of the negated terms, see coop_lin)
__device__ __forceinline__ Fp acc_reduce(Acc13 a, uint32_t extra) {
  uint32_t k20p[13];
#pragma unroll
  for (int i = 0; i < 13; ++i) k20p[i] = k20p_limb(i);
  k20p[0] += extra;          // 0xaab00000 + extra: no carry
  asm_acc_add13(a.l, k20p);  // now 0 <= a < 2^21 p
  // q ~ a / p from the top 96 bits in double precision (|error| < 1); q - 1 makes
  // a - (q - 1) p land in [0, 3p)
  double d = (double)a.l[12] * 18446744073709551616.0 + (double)a.l[11] * 4294967296.0 + (double)a.l[10];
  uint32_t q = (uint32_t)(d * 0x1.3b06ba5e7993dp-61);
  q = q > 0u ? q - 1u : 0u;
  uint32_t qp[13], carry = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint64_t v = (uint64_t)p_limb(i) * q + carry;
    qp[i] = (uint32_t)v;
    carry = (uint32_t)(v >> 32);
  }
  qp[12] = carry;
  asm_acc_sub13(a.l, qp);
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.l[i] = a.l[i];
  return r;
}

// canonical form of a lazy value x < 3p
__device__ __forceinline__ Fp fp_canon3(const Fp& x) {
  const uint32_t pl[12] = {BLS_P_LIMBS};
  Fp d1, d2;
  const uint32_t b1 = asm_sub12(d1.l, x.l, pl);
  const uint32_t b2 = asm_sub12(d2.l, d1.l, pl);
  return b1 ? x : (b2 ? d1 : d2);
}

__device__ __forceinline__ bool fp_is_zero_lazy(const Fp& x) { return fp_is_zero(fp_canon3(x)); }

// sum_k cf[k] * slot[refs[k]] mod p over n <= 8 terms.  refs index the block's LDS
// slot array (frame, then the constant bank at COOP_FRAME).  Branch-free up to the
// wave's largest n (loop bound wave-uniform; a lane's unused term has coefficient 0):
// each term is 12 multiply-adds of its limbs, complemented for c < 0, by |c| into 64-bit
// limb columns (8 x 2^32 x 2^15 < 2^50: no carries until the end), then one carry pass.
// A negated term adds |c| (2^384 - 1 - x) = -|c| x + |c| (2^384 - 1): the 2^384 part
// leaves limb 12, the -|c| goes to the reduction bias.  (Round 3 formed every product
// x |c| as a 13-limb number and added it with a carry chain: ~62 instructions per term
// against ~26 here.)
// The unreduced sum as a 13-limb two's-complement accumulator; returns the sum of |c|
// over the negated terms (acc_reduce's bias)
__device__ __forceinline__ uint32_t coop_lin_acc(const uint16_t (&refs)[8], const int16_t (&cf)[8], int n,
                                                 int nmax, const LdsU4* slots, Acc13& acc) {
  uint64_t col[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) col[i] = 0;
  uint32_t negs = 0;  // sum of |c| over the negated terms
  // (terms past a lane's n have coefficient 0 and slot 0 in the table: no masking; the
  // next term's LDS reads issued before this term's multiply-adds measured slower,
  // profiles/r05_ab_coop_prefetch.json)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k >= nmax) break;
    const int c = cf[k];
    const uint32_t mask = c < 0 ? 0xffffffffu : 0u;
    const uint32_t m = c < 0 ? (uint32_t)(-c) : (uint32_t)c;
    negs += mask & m;
    const Fp x = lds_load_fp(slots, refs[k]);
#pragma unroll
    for (int i = 0; i < 12; ++i) col[i] += (uint64_t)(x.l[i] ^ mask) * m;
  }
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    acc.l[i] = (uint32_t)col[i];
    col[i + 1] += col[i] >> 32;
  }
  acc.l[11] = (uint32_t)col[11];
  acc.l[12] = (uint32_t)(col[11] >> 32) - negs;  // two's complement: the -|c| 2^384 of the negated terms
  return negs;
}

// nmax / single: the step's wave-uniform largest term count and "one +1 term on every
// lane" (CoopOp ma / mb / flags, scalar registers)
__device__ __forceinline__ Fp coop_lin(const uint16_t (&refs)[8], const int16_t (&cf)[8], int n, int nmax,
                                       bool single, const LdsU4* slots) {
  if (single) return lds_load_fp(slots, refs[0]);
  Acc13 acc;
  const uint32_t negs = coop_lin_acc(refs, cf, n, nmax, slots, acc);
  return acc_reduce(acc, negs);
}

// the value of lane ^ 1 / lane ^ 2 (DPP quad_perm [1,0,3,2] / [2,3,0,1]; every lane of the
// wave must take part)
__device__ __forceinline__ uint32_t coop_pair_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t coop_half_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
}

// One lane's op of one step as fetched: the 80-byte CoopOp as 20 raw dwords, loaded
// with five global (not flat) dwordx4 loads.  Fields are decoded only where the
// step that owns the op executes, so the loads of the next step's op stay in flight
// (vmcnt only; flat loads would also hold lgkmcnt and stall every LDS wait).
struct CoopOpRaw {
  bls_u32x4 w[4];
  bls_u32x2 t;  // dwords 16, 17 (cb[4..7]); the 8 pad bytes are never loaded
};
typedef __attribute__((address_space(1))) const bls_u32x4 GlobU4;
typedef __attribute__((address_space(1))) const bls_u32x2 GlobU2;

// Unconditional (every lane, every step), so the compiler can count the loads in
// flight with vmcnt instead of waiting for them at a control-flow merge.
__device__ __forceinline__ void coop_fetch(CoopOpRaw& u, const GlobU4* base, uint32_t step, int lane) {
  const GlobU4* src = base + ((size_t)step * COOP_LANES + lane) * 5;
#pragma unroll
  for (int k = 0; k < 4; ++k) u.w[k] = src[k];
  u.t = *(const GlobU2*)(src + 4);
}

// dword k (0..19) of the raw op
__device__ __forceinline__ uint32_t op_word(const CoopOpRaw& u, int k) { return k < 16 ? u.w[k >> 2][k & 3] : u.t[k & 1]; }

// Decoded view of a raw op (CoopOp layout: out u16, kind u8, na u8 | nb u8 ... |
// a[8] u16 @8 | b[8] u16 @24 | ca[8] i16 @40 | cb[8] i16 @56)
struct CoopOpView {
  uint32_t out, kind, na, nb;
  int ma, mb;        // wave-uniform (readfirstlane)
  bool sa, sb;
  int lgp, lgl;      // log2 of the product / combination lane-group sizes (wave-uniform)
  uint16_t a[8], b[8];
  int16_t ca[8], cb[8];
};

__device__ __forceinline__ CoopOpView coop_decode(const CoopOpRaw& u) {
  CoopOpView v;
  const uint32_t w0 = op_word(u, 0), w1 = op_word(u, 1);
  v.out = w0 & 0xffffu;
  v.kind = (w0 >> 16) & 0xffu;
  v.na = w0 >> 24;
  v.nb = w1 & 0xffu;
  const uint32_t s1 = __builtin_amdgcn_readfirstlane(w1);  // every lane carries the same bytes 1-3
  v.ma = (int)((s1 >> 8) & 0xffu);
  v.mb = (int)((s1 >> 16) & 0xffu);
  v.sa = (s1 >> 24) & 1u;
  v.sb = (s1 >> 25) & 1u;
  v.lgp = (int)((s1 >> 26) & 3u);
  v.lgl = (int)((s1 >> 28) & 3u);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t wa = op_word(u, 2 + k), wb = op_word(u, 6 + k), wca = op_word(u, 10 + k), wcb = op_word(u, 14 + k);
    v.a[2 * k] = (uint16_t)wa;
    v.a[2 * k + 1] = (uint16_t)(wa >> 16);
    v.b[2 * k] = (uint16_t)wb;
    v.b[2 * k + 1] = (uint16_t)(wb >> 16);
    v.ca[2 * k] = (int16_t)wca;
    v.ca[2 * k + 1] = (int16_t)(wca >> 16);
    v.cb[2 * k] = (int16_t)wcb;
    v.cb[2 * k + 1] = (int16_t)(wcb >> 16);
  }
  return v;
}

// Wave-local step boundary.  A block is one wavefront: its LDS operations complete
// in issue order, so a step needs only its reads to have landed before the writes
// (and the compiler not to move LDS accesses across) -- no s_barrier.
__device__ __forceinline__ void coop_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One step for this lane: gather, product, then (after the wave's gathers) write.
// TIMED (the probe, bls_gpu_coop_probe): lane 0 stamps s_memtime at the point `mark`
// names -- 0: compute done (before the fence), 1: op decoded, 2: operand a summed,
// 3: operand b summed (product steps), 4: product done.
// W wavefronts per task (a block of 64 W lanes, program steps of 64 W ops): the step
// boundaries are block barriers then
template <int W>
__device__ __forceinline__ void coop_task_sync() {
  if (W == 1) coop_wave_sync();
  else __syncthreads();
}

template <bool TIMED, int W = 1>
__device__ __forceinline__ void coop_step(const CoopOpRaw& raw, LdsU4* slots, uint32_t* flag, uint64_t* stamp,
                                          uint32_t mark = 0) {
  const CoopOpView op = coop_decode(raw);
  if (TIMED && mark == 1 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memtime();
  Fp r = fp_zero();
  if (op.lgp == 0 && op.lgl == 0) {  // one lane per op
    if (op.kind != 0) {
      r = coop_lin(op.a, op.ca, op.na, op.ma, op.sa, slots);
      if (TIMED && mark == 2 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memtime();
      if (op.kind == COOP_MUL) {
        const Fp rb = coop_lin(op.b, op.cb, op.nb, op.mb, op.sb, slots);
        if (TIMED && mark == 3 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memtime();
        r = fp_mul_lazy(r, rb);
        if (TIMED && mark == 4 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memtime();
      }
    }
  } else {
    // lane groups (tools/gen_coop.py lane_entries): every lane sums its part of its
    // operand unreduced; the parts of one operand are added by DPP butterflies (lanes
    // ^1, then ^2, within the aligned group: a combination's whole group, a product
    // operand's half of its group); one reduction; a product group's halves then swap
    // their operands and every lane of it multiplies (the product is symmetric)
    const bool grp = op.kind == COOP_GRP_A || op.kind == COOP_GRP_B;
    const int lv = grp ? op.lgp - 1 : (op.kind == COOP_LIN ? op.lgl : 0);
    const int levels = op.lgp - 1 > op.lgl ? op.lgp - 1 : op.lgl;
    Acc13 acc, oth;
    uint32_t negs = coop_lin_acc(op.a, op.ca, op.kind ? (int)op.na : 0, op.ma, slots, acc);
    if (levels > 0) {
#pragma unroll
      for (int i = 0; i < 13; ++i) oth.l[i] = coop_pair_swap(acc.l[i]);
      const uint32_t on = coop_pair_swap(negs);
      if (lv > 0) {
        asm_acc_add13(acc.l, oth.l);
        negs += on;
      }
    }
    if (levels > 1) {
#pragma unroll
      for (int i = 0; i < 13; ++i) oth.l[i] = coop_half_swap(acc.l[i]);
      const uint32_t on = coop_half_swap(negs);
      if (lv > 1) {
        asm_acc_add13(acc.l, oth.l);
        negs += on;
      }
    }
    r = acc_reduce(acc, negs);
    if (TIMED && mark == 2 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memtime();
    if (op.kind == COOP_MUL) r = fp_mul_lazy(r, coop_lin(op.b, op.cb, op.nb, op.mb, op.sb, slots));
    if (op.lgp > 0) {
      Fp o;
      if (op.lgp == 1) {
#pragma unroll
        for (int i = 0; i < 12; ++i) o.l[i] = coop_pair_swap(r.l[i]);
      } else {
#pragma unroll
        for (int i = 0; i < 12; ++i) o.l[i] = coop_half_swap(r.l[i]);
      }
      if (grp) r = fp_mul_lazy(r, o);
    }
    if (TIMED && mark == 4 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memtime();
  }
  if (TIMED && mark == 0 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memtime();
  coop_task_sync<W>();
  if (op.kind != 0 && op.out != COOP_OUT_NONE) {  // (a group writes from its first lane)
    if (op.out >= COOP_OUT_ZSET) {  // zero-check: bit 0 (0xFFFF) or bit s of packed set s (0xFFF0 + s)
      if (fp_is_zero_lazy(r)) atomicOr(flag, op.out == COOP_OUT_ZCHECK ? 1u : 1u << (op.out - COOP_OUT_ZSET));
    } else {
      lds_store_fp(slots, op.out, r);
    }
  }
  coop_task_sync<W>();
}

// Run one program on this block's frame.  cbank: the constant bank staged in LDS
// (coop_stage_consts).  *flag (LDS) is set when a zero-check op sees zero.  Two op
// buffers alternate: step s computes from one while step s + 1's ops load into the
// other.
// W: wavefronts per task; a W-wavefront program's step is W consecutive 64-op records
// (tools/gen_coop.py emit, programs named *_w2), lane threadIdx.x reads op threadIdx.x
template <bool TIMED, int W = 1>
__device__ __forceinline__ void coop_run_body(const CoopEnv& env, CoopProg pg, Fp* frame, uint32_t* flag,
                                              uint64_t* stamps) {
  const int lane = threadIdx.x;
  const GlobU4* base = (const GlobU4*)(const void*)env.ops;
  if (pg.n == 0) return;
  LdsU4* slots = (LdsU4*)frame;
  CoopOpRaw A, B;
  const uint32_t mark = TIMED && stamps ? (uint32_t)stamps[0] : 0u;  // the probe's stamp point
  const uint32_t last = pg.first + W * (pg.n - 1);
  coop_fetch(A, base, pg.first, lane);
  for (uint32_t s = 0; s < pg.n; s += 2) {
    const uint32_t g = pg.first + W * s;
    if (TIMED && lane == 0) stamps[2 * s] = __builtin_amdgcn_s_memtime();
    coop_fetch(B, base, g + W <= last ? g + W : last, lane);
    coop_step<TIMED, W>(A, slots, flag, stamps ? stamps + 2 * s + 1 : nullptr, mark);
    if (s + 1 >= pg.n) break;
    if (TIMED && lane == 0) stamps[2 * s + 2] = __builtin_amdgcn_s_memtime();
    coop_fetch(A, base, g + 2 * W <= last ? g + 2 * W : last, lane);
    coop_step<TIMED, W>(B, slots, flag, stamps ? stamps + 2 * s + 3 : nullptr, mark);
  }
  if (TIMED && lane == 0) stamps[2 * pg.n] = __builtin_amdgcn_s_memtime();
}

// Out of line: one copy of the interpreter per code object.  Its register count
// (256 with the default budget) then caps every caller at 2 wavefronts per SIMD.
template <bool TIMED>
__device__ __noinline__ void coop_run_t(const CoopEnv& env, CoopProg pg, Fp* frame, const Fp* cbank,
                                        uint32_t* flag, uint64_t* stamps) {
  coop_run_body<TIMED>(env, pg, frame, flag, stamps);
}

__device__ __forceinline__ void coop_run(const CoopEnv& env, CoopProg pg, Fp* frame, const Fp* cbank,
                                         uint32_t* flag) {
  coop_run_t<false>(env, pg, frame, cbank, flag, nullptr);
}

// a two-wavefront program (both wavefronts of the block call it)
__device__ __noinline__ void coop_run2_t(const CoopEnv& env, CoopProg pg, Fp* frame, uint32_t* flag) {
  coop_run_body<false, 2>(env, pg, frame, flag, nullptr);
}

// copy the constant bank into LDS (once per block)
__device__ __forceinline__ void coop_stage_consts(const CoopEnv& env, Fp* cbank) {
  for (uint32_t k = threadIdx.x; k < env.n_consts; k += COOP_LANES) lds_store_fp(cbank, k, env.consts[k]);
  __syncthreads();
}

// lane 0 inverts frame[in] into frame[out]; the wavefront (the block) waits
__device__ __forceinline__ void coop_invert(Fp* frame, int in, int out) {
  if (threadIdx.x == 0) lds_store_fp(frame, out, fp_inv_gcd(fp_canon3(lds_load_fp(frame, in))));
  coop_wave_sync();
}

// cooperative copies between global memory and the frame (n slots)
__device__ __forceinline__ void coop_load(Fp* frame, int slot, const Fp* src, int n) {
  for (int k = threadIdx.x; k < n; k += COOP_LANES) lds_store_fp(frame, slot + k, src[k]);
  __syncthreads();
}

__device__ __forceinline__ bool coop_is_zero(const Fp* frame, int slot, int n) {
  bool z = true;
  for (int k = 0; k < n; ++k) z = z && fp_is_zero_lazy(lds_load_fp(frame, slot + k));
  return z;
}

// canonical value of a frame slot (for export to global memory / exact compares)
__device__ __forceinline__ Fp coop_get(const Fp* frame, int slot) { return fp_canon3(lds_load_fp(frame, slot)); }

}  // namespace bls
