// Signature stage: compressed G2 decode + psi(P) == [x]P subgroup check (one lane per set).
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_sig(PipeBufs b) { stage_sig(b, blockIdx.x * BLS_BLOCK + threadIdx.x); }

hipError_t launch_k_sig(const PipeBufs& b, hipStream_t s) {
  k_sig<<<bls_grid_for(b.n_sets), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
