// Standalone hash_to_G2 entry point (bls_gpu_hash_to_g2), one lane per message.
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_hash_to_g2(const uint8_t* msgs, uint32_t n, uint8_t* out192) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  msg_words_from_bytes(msgs + 32ull * i, w);
  g2_serialize192(hash_to_g2(w), out192 + 192ull * i);
}

hipError_t launch_k_hash_to_g2(const uint8_t* msgs, uint32_t n, uint8_t* out192, hipStream_t s) {
  k_hash_to_g2<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(msgs, n, out192);
  return hipGetLastError();
}
