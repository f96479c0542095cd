// hash_to_G2 stage (one lane per set) and the standalone hash_to_G2 entry point.
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_h2c(PipeBufs b) { stage_h2c(b, blockIdx.x * BLS_BLOCK + threadIdx.x); }

__global__ __launch_bounds__(BLS_BLOCK) void k_hash_to_g2(const uint8_t* msgs, uint32_t n, uint8_t* out192) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  msg_words_from_bytes(msgs + 32ull * i, w);
  g2_serialize192(hash_to_g2(w), out192 + 192ull * i);
}

hipError_t launch_k_h2c(const PipeBufs& b, hipStream_t s) {
  k_h2c<<<bls_grid_for(b.n_sets), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
hipError_t launch_k_hash_to_g2(const uint8_t* msgs, uint32_t n, uint8_t* out192, hipStream_t s) {
  k_hash_to_g2<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(msgs, n, out192);
  return hipGetLastError();
}
