// Field self-test and Fp-product probes: canonical-byte Fp products (parity against
// the oracle) and a dependent chain of Montgomery products per lane (latency when
// one wave runs alone, throughput when every CU is busy).
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_fp_mul_test(const uint8_t* a, const uint8_t* b, uint32_t n,
                                                           uint8_t* out) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  Fp x = fp_to_mont(fp_from_be48(a + 48ull * i));
  Fp y = fp_to_mont(fp_from_be48(b + 48ull * i));
  // equal operands go through the dedicated squaring
  fp_to_be48(fp_from_mont(fp_eq(x, y) ? fp_sqr(x) : fp_mul(x, y)), out + 48ull * i);
}

__global__ __launch_bounds__(BLS_BLOCK) void k_fpm_chain(Fp* io, uint32_t iters) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  Fp a = io[2 * i], b = io[2 * i + 1];
  for (uint32_t k = 0; k < iters; ++k) a = fp_mul(a, b);
  io[2 * i] = a;
}

hipError_t launch_k_fp_mul_test(const uint8_t* a, const uint8_t* b, uint32_t n, uint8_t* out, hipStream_t s) {
  k_fp_mul_test<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(a, b, n, out);
  return hipGetLastError();
}
hipError_t launch_k_fpm_chain(Fp* io, uint32_t lanes, uint32_t iters, hipStream_t s) {
  k_fpm_chain<<<lanes / BLS_BLOCK, BLS_BLOCK, 0, s>>>(io, iters);
  return hipGetLastError();
}
