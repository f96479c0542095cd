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

// Signature.fromBytes(bytes, affine, validate) for n compressed signatures: the same
// decoder the verify path runs (g2_decompress96), then the exact G2 membership test.
__global__ __launch_bounds__(BLS_BLOCK) void k_g2_decompress(const uint8_t* in96, uint32_t n, int validate,
                                                             uint8_t* out192, int32_t* codes) {
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  G2A a;
  int32_t code = g2_decompress96(in96 + 96ull * i, a);
  if (code == BLS_OK && validate && !a.inf && !g2_in_subgroup(a)) code = BLS_POINT_NOT_IN_GROUP;
  if (code != BLS_OK) {
    a.inf = true;
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  g2_serialize192(a, out192 + 192ull * i);
  codes[i] = code;
}

hipError_t launch_k_g2_decompress(const uint8_t* in96, uint32_t n, int validate, uint8_t* out192, int32_t* codes,
                                  hipStream_t s) {
  k_g2_decompress<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(in96, n, validate, out192, codes);
  return hipGetLastError();
}
