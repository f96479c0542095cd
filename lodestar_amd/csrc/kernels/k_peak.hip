// VALU integer roofline probe: back-to-back v_mad_u64_u32 (32x32+64 -> 64), the
// instruction every Fp Montgomery product is built from (288 per CIOS product).
// 8 independent chains per lane for ILP; the grid fills every CU at 8 waves/SIMD.
#include "../launchers.hpp"

__global__ __launch_bounds__(256) void k_mad_peak(uint64_t* out, uint32_t iters, uint32_t seed) {
  uint32_t b = (threadIdx.x + 1u) * 2654435761u ^ seed;
  uint64_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = (uint64_t)(b + k) << 7;
  for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = (uint64_t)(uint32_t)acc[k] * b + acc[k];
    }
  }
  uint64_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= acc[k];
  if (x == 0x9e3779b97f4a7c15ull) out[blockIdx.x] = x;  // keep the chains live
}

hipError_t launch_k_mad_peak(uint64_t* out, uint32_t blocks, uint32_t iters, hipStream_t s) {
  k_mad_peak<<<blocks, 256, 0, s>>>(out, iters, 12345u);
  return hipGetLastError();
}
