// Random-scalar stage: r_i * pk_i (G1) and r_i * sig_i (G2), one lane per set.
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_scale(PipeBufs b) { stage_scale(b, blockIdx.x * BLS_BLOCK + threadIdx.x); }

hipError_t launch_k_scale(const PipeBufs& b, hipStream_t s) {
  k_scale<<<bls_grid_for(b.n_sets), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
