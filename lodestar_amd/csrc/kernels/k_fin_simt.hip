// SIMT final exponentiations: one lane per task, for a failing pass's MANY tasks.
//
//   k_chunk_simt  one lane per chunk of batchable requests: FE(prod f_i of its sets x its
//                 units x its signature-sum pairing) == 1 (worker.ts:56-88)
//   k_indiv_simt  one lane per request verified alone (a failed chunk's, or a
//                 non-batchable one; worker.ts:91-98): FE(prod f_i x its own signature-sum
//                 pairing) == 1, or the request's product only for group testing
//
// The same tasks as k_chunk_coop / k_indiv_coop (kernels/k_fin.hip, one 64-lane
// wavefront per task running the interpreted final exponentiation), with the same
// verdicts (bls/pairing.hpp final_exponentiation is the function both compute;
// test_gpu_parity runs both).  A cooperative task holds a SIMD for the ~1.4 ms of one
// final exponentiation; here one wavefront finishes 64 tasks in a few ms, ~10x less
// device time per task -- what a failing pass at the plateau (cfg4 per-set requests:
// ~500 chunk checks and ~1,300 requests alone per 8,192-set pass) pays for, while the
// cooperative form stays the choice for a few tasks, whose latency is the call's
// (launch_k_chunk_fe / launch_k_indiv_fe pick by the task count, $BLS_FE_SIMT_MIN).
#define BLS_FP_D28 1
#include <stdlib.h>

#include "../launchers.hpp"
#include "bls/pairing.hpp"

using namespace bls;

namespace {

// The final exponentiation with ONE Fp12 in registers at a time: every other operand is
// read from the task's four slots in device memory (save + 4 t, not the runtime's per-
// queue scratch, which admission prices -- a register-resident form spilled 5.7-7.7 KB
// per lane).  The steps and their order are pairing.hpp's final_exponentiation, so the
// value is the same, e(P, Q)^3.

// a * m (CONJ: a * conj(m)), m in memory: Karatsuba over Fp6 (field.hpp fp12_mul)
template <bool CONJ>
__device__ __forceinline__ Fp12 mul12m(const Fp12& a, const Fp12* m) {
  const Fp6 t0 = fp6_mul(a.c0, m->c0);
  Fp6 t1 = fp6_mul(a.c1, m->c1);
  const Fp6 mc1 = CONJ ? fp6_neg(m->c1) : m->c1;
  const Fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(m->c0, mc1)), t0), CONJ ? fp6_neg(t1) : t1);
  if (CONJ) t1 = fp6_neg(t1);
  return Fp12{fp6_add(t0, fp6_mul_v(t1)), c1};
}

// Granger-Scott squaring (field.hpp fp12_cyclotomic_sqr, inlined)
__device__ __forceinline__ Fp12 cyc_sqr(const Fp12& f) {
  Fp2 a0, a1, b0, b1, d0, d1;
  fp4_sqr(f.c0.c0, f.c1.c1, a0, a1);
  fp4_sqr(f.c1.c0, f.c0.c2, b0, b1);
  fp4_sqr(f.c0.c1, f.c1.c2, d0, d1);
  Fp12 r;
  r.c0.c0 = fp2_add(fp2_dbl(fp2_sub(a0, f.c0.c0)), a0);
  r.c1.c1 = fp2_add(fp2_dbl(fp2_add(a1, f.c1.c1)), a1);
  const Fp2 xd1 = fp2_mul_xi(d1);
  r.c1.c0 = fp2_add(fp2_dbl(fp2_add(xd1, f.c1.c0)), xd1);
  r.c0.c2 = fp2_add(fp2_dbl(fp2_sub(d0, f.c0.c2)), d0);
  r.c0.c1 = fp2_add(fp2_dbl(fp2_sub(b0, f.c0.c1)), b0);
  r.c1.c2 = fp2_add(fp2_dbl(fp2_add(b1, f.c1.c2)), b1);
  return r;
}

// *out = base^x = conj(base^|x|), base in the cyclotomic subgroup (pairing.hpp
// fp12_cyclotomic_exp_x); base is read from memory at each of |x|'s set bits
__device__ __noinline__ void exp_x_m(const Fp12* base, Fp12* out) {
  Fp12 r = *base;
  const uint64_t X = BLS_X_ABS;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    r = cyc_sqr(r);
    if ((X >> i) & 1ull) r = mul12m<false>(r, base);
  }
  *out = fp12_conj(r);
}

// FE(F) == 1 (pairing.hpp final_exponentiation), S = the task's four slots
__device__ __forceinline__ bool fe_is_one(Fp12 F, Fp12* S) {
  // easy part: t = conj(F) / F, then t^(p^2 + 1)
  S[0] = fp12_conj(F);
  Fp12 t = mul12m<false>(fp12_inv(F), &S[0]);
  S[1] = t;
  t = mul12m<false>(fp12_frob2(t), &S[1]);
  // hard part (HHT): t^((x-1)^2 (x+p)(x^2+p^2-1)) * t^3
  S[0] = t;
  S[3] = mul12m<false>(cyc_sqr(t), &S[0]);                 // t^3
  exp_x_m(&S[0], &S[1]);
  S[0] = mul12m<true>(S[1], &S[0]);                        // a = t^(x-1)
  exp_x_m(&S[0], &S[1]);
  S[0] = mul12m<true>(S[1], &S[0]);                        // a = t^((x-1)^2)
  exp_x_m(&S[0], &S[1]);
  S[2] = mul12m<false>(fp12_frob(S[0]), &S[1]);            // b = a^(x+p)
  exp_x_m(&S[2], &S[0]);
  exp_x_m(&S[0], &S[1]);                                   // c = b^(x^2)
  Fp12 c = mul12m<false>(fp12_frob2(S[2]), &S[1]);         // c b^(p^2)
  S[0] = c;
  c = mul12m<true>(S[0], &S[2]);                           // ... b^-1 (conj: b is unitary)
  return fp12_is_one(mul12m<false>(c, &S[3]));             // ... t^3
}

}  // namespace

__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_chunk_simt(PipeBufs b,
                                                                                                  Fp12* save) {
  BLS_TAIL_PRIO();
  const uint32_t c = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (c >= b.n_chunks) return;
  const uint32_t beg = b.chunk_off[c], end = b.chunk_off[c + 1];
  for (uint32_t k = beg; k < end; ++k)
    if (b.req_status[b.chunk_reqs[k]] != BLS_OK) {
      b.chunk_ok[c] = 0;  // the batch would throw -> retry every request (worker.ts:81-87)
      return;
    }
  Fp12 F = fp12_one();
  for (uint32_t k = beg; k < end; ++k) {
    const uint32_t r = b.chunk_reqs[k];
    for (uint32_t i = b.req_off[r]; i < b.req_off[r + 1]; ++i) {
      // a live set paired in its Miller-loop unit has f_i = 1 (k_chunk_coop likewise)
      if (b.set_unit && b.set_unit[i] != UNIT_NONE && b.chain_live[i]) continue;
      F = mul12m<false>(F, &b.f[i]);
    }
  }
  if (b.sigagg) F = mul12m<false>(F, &b.f[b.n_sets + c]);  // ML(-g1, sum of the chunk's r sig)
  if (b.unit_off)
    for (uint32_t u = b.unit_off[c]; u < b.unit_off[c + 1]; ++u) F = mul12m<false>(F, &b.f[b.unit_base + u]);
  b.chunk_ok[c] = fe_is_one(F, save + 4ull * c) ? 1 : 0;
}

__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_indiv_simt(PipeBufs b,
                                                                                                  GroupBufs gb,
                                                                                                  Fp12* save) {
  BLS_TAIL_PRIO();
  const uint32_t t = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (t >= b.n_indiv) return;
  const uint32_t r = b.indiv_reqs[t];
  const int32_t code = b.req_status[r];
  if (code != BLS_OK) {
    b.indiv_verdict[t] = -code;
    return;
  }
  Fp12 F = fp12_one();
  const uint32_t stride = b.fold > 1 ? b.fold : 1u;  // f's pre-multiplied in groups by k_fold
  for (uint32_t i = b.req_off[r]; i < b.req_off[r + 1]; i += stride) F = mul12m<false>(F, &b.f[i]);
  if (b.sigagg && (t < gb.n_direct || !gb.sum_f)) F = mul12m<false>(F, &b.f[b.indiv_vbase + t]);  // its own sum
  if (t >= gb.n_direct) {  // group-tested: the product only (k_group_coop)
    gb.f[t] = F;
    b.indiv_verdict[t] = 2;
    return;
  }
  b.indiv_verdict[t] = fe_is_one(F, save + 4ull * t) ? 1 : 0;
}

// the task count from which a failing pass's final exponentiations run one lane per
// task ($BLS_FE_SIMT_MIN; default 0 = off: at 256 the cfg4 per-set-request slice ran
// 1.04M vs 1.15M sets/s steady and the cfg5 slice 2.56M vs 2.83M -- a lane's ~8k
// dependent Fp products take ~8 ms, and those passes wait on the tail's latency, not on
// device time; profiles/r06_ab_fe_simt.json)
uint32_t fe_simt_min() {
  static const uint32_t v = [] {
    const char* e = getenv("BLS_FE_SIMT_MIN");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : 0u;
  }();
  return v;
}

// save: 4 Fp12 per task (chunks / requests)
hipError_t launch_k_chunk_simt(const PipeBufs& b, Fp12* save, hipStream_t s) {
  if (b.n_chunks == 0) return hipSuccess;
  k_chunk_simt<<<bls_grid_for(b.n_chunks), BLS_BLOCK, 0, s>>>(b, save);
  return hipGetLastError();
}

hipError_t launch_k_indiv_simt(const PipeBufs& b, const GroupBufs& g, Fp12* save, hipStream_t s) {
  if (b.n_indiv == 0) return hipSuccess;
  k_indiv_simt<<<bls_grid_for(b.n_indiv), BLS_BLOCK, 0, s>>>(b, g, save);
  return hipGetLastError();
}
