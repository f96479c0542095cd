// Single-lane pre-stage of the verify path (pipeline.hpp stage_pre): for every
// distinct signing root the two SSWU points on E2' (expand_message_xmd + hash_to_field + SSWU, two Fp
// exponentiations each) and the signature decompression.  Lanes [0, 2u) map,
// lanes [2u, 2u + n) decode, so each wavefront runs one kind of work; k_qdup then
// hands each set its root's points.
#define BLS_FP_D28 1  // 28-bit-digit Montgomery product (bls/field.hpp)
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_pre(PipeBufs b) { stage_pre(b, blockIdx.x * BLS_BLOCK + threadIdx.x); }

__global__ __launch_bounds__(BLS_BLOCK) void k_qdup(PipeBufs b) { stage_qdup(b, blockIdx.x * BLS_BLOCK + threadIdx.x); }

hipError_t launch_k_pre(const PipeBufs& b, hipStream_t s) {
  k_pre<<<bls_grid_for(pre_lanes(b)), BLS_BLOCK, 0, s>>>(b);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !b.msg_rep) return e;
  k_qdup<<<bls_grid_for(8 * b.n_sets), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
