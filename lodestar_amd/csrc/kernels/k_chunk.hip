// Batch stage: one lane per chunk of >= 16 batchable requests (product, ML(-g1, S), final exponentiation).
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_chunk(PipeBufs b) { stage_chunk(b, blockIdx.x * BLS_BLOCK + threadIdx.x); }

hipError_t launch_k_chunk(const PipeBufs& b, hipStream_t s) {
  k_chunk<<<bls_grid_for(b.n_chunks), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
