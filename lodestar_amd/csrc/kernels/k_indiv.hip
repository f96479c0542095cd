// Fallback stage: one lane per request verified on its own.
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_indiv(PipeBufs b) { stage_indiv(b, blockIdx.x * BLS_BLOCK + threadIdx.x); }

hipError_t launch_k_indiv(const PipeBufs& b, hipStream_t s) {
  k_indiv<<<bls_grid_for(b.n_indiv), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
