// Miller-loop stage: f_i = ML(r_i pk_i, H(m_i)), one lane per set.
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_miller(PipeBufs b) { stage_miller_set(b, blockIdx.x * BLS_BLOCK + threadIdx.x); }

hipError_t launch_k_miller(const PipeBufs& b, hipStream_t s) {
  k_miller<<<bls_grid_for(b.n_sets), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
