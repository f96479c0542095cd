// Single-lane pre-stage of the verify path (pipeline.hpp stage_pre): for every
// distinct signing root the two SSWU points on E2' (expand_message_xmd + hash_to_field + SSWU, two Fp
// exponentiations each) and the signature decompression.  Lanes [0, 2u) map, lanes
// [base, base + n) decode from the next wavefront boundary (pipeline.hpp
// pre_decode_base), so each wavefront runs one kind of work; k_qdup then hands each set
// its root's points.
#define BLS_FP_D28 1  // 28-bit-digit Montgomery product (bls/field.hpp)
#include "../launchers.hpp"

using namespace bls;

// Per-set path (k_pset): RP = [s] pk and RG = [s] g1 for the set's batch scalar s (GLV:
// curve.hpp jac_mul_glv, the scalar convention of k_chain and k_msm), two lanes per set
// after the SSWU and decode lanes (from a wavefront boundary, so no wavefront mixes the
// kinds).  The ~0.9 ms GLV chain runs beside the ~1.4 ms SSWU chains on other CUs: off
// the small call's critical path (in k_pset's second wavefront it slowed the first by
// 0.35 ms, profiles/r04_ab_pset_rpoints.json).  RP at infinity (a public key of small
// order) sends the set to the exact path.
__device__ __noinline__ void pre_rpts(const PipeBufs& b, uint32_t j) {
  const uint32_t i = j >> 1, which = j & 1u;
  if (b.pk_status[i] != BLS_OK || jac_is_inf(b.pk[i])) return;  // errors out; f_i unused
  const G1J p = which == 0 ? b.pk[i] : jac_from_aff(g1_generator());
  uint32_t a, c;
  glv_split(set_scalar(b.seed, b.scalar_base + i), a, c);
  const G1J q = jac_mul_glv<Fp>(p, a, c, b.rtab1 + 15ull * j);
  b.rpts[j] = q;
  if (which == 0 && jac_is_inf(q)) b.set_flag[i] = 1u;
}

__device__ __forceinline__ uint32_t pre_rpts_base(const PipeBufs& b) {
  return (pre_lanes(b) + BLS_BLOCK - 1) / BLS_BLOCK * BLS_BLOCK;
}

// three wavefronts per SIMD (168 VGPRs, 1,664 B/lane of scratch: 327 MiB per queue, under
// k_chain's 337): cfg2 3.85-3.87M vs 3.79-3.81M sets/s at two per SIMD (255 VGPRs), the
// k_pre stage 9.0 vs 10.8-11.9 ms, p50 @128 level; one per SIMD 3.61M; four would reserve
// 570 MiB per queue, past the admission budget at 16 contexts (profiles/r06_ab_pre_occ.json)
#ifndef BLS_PRE_WAVES
#define BLS_PRE_WAVES 3
#endif
__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(BLS_PRE_WAVES))) void k_pre(PipeBufs b) {
  const uint32_t t = blockIdx.x * BLS_BLOCK + threadIdx.x;
  const uint32_t base = pre_rpts_base(b);
  if (t < base) stage_pre(b, t);
  else if (b.rpts && t < base + 2 * b.n_sets) pre_rpts(b, t - base);
}

__global__ __launch_bounds__(BLS_BLOCK) void k_qdup(PipeBufs b) { stage_qdup(b, blockIdx.x * BLS_BLOCK + threadIdx.x); }

hipError_t launch_k_pre(const PipeBufs& b, hipStream_t s) {
  const uint32_t lanes = (pre_lanes(b) + BLS_BLOCK - 1) / BLS_BLOCK * BLS_BLOCK + (b.rpts ? 2 * b.n_sets : 0u);
  k_pre<<<bls_grid_for(lanes), BLS_BLOCK, 0, s>>>(b);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !b.msg_rep) return e;
  k_qdup<<<bls_grid_for(8 * b.n_sets), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
