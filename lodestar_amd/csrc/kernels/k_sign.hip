// Fixture helpers: sk -> pk (G1) and sign = sk * hash_to_G2(msg) (G2).  Not on the verify path.
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_sk_to_pk(const uint8_t* sks, uint32_t n, uint8_t* out48) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  scalar_words_from_be32(sks + 32ull * i, k);
  g1_compress48(jac_to_aff(aff_mul_u256(g1_generator(), k)), out48 + 48ull * i);
}

__global__ __launch_bounds__(BLS_BLOCK) void k_sign(const uint8_t* sks, const uint8_t* msgs, uint32_t n,
                                                    uint8_t* out96) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8], w[8];
  scalar_words_from_be32(sks + 32ull * i, k);
  msg_words_from_bytes(msgs + 32ull * i, w);
  g2_compress96(jac_to_aff(aff_mul_u256(hash_to_g2(w), k)), out96 + 96ull * i);
}

hipError_t launch_k_sk_to_pk(const uint8_t* sks, uint32_t n, uint8_t* out48, hipStream_t s) {
  k_sk_to_pk<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(sks, n, out48);
  return hipGetLastError();
}
hipError_t launch_k_sign(const uint8_t* sks, const uint8_t* msgs, uint32_t n, uint8_t* out96, hipStream_t s) {
  k_sign<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(sks, msgs, n, out96);
  return hipGetLastError();
}
