// Design probes (bls_gpu_kernel_probe): kernels that time one formulation of a hot
// stage on synthetic operands, so a re-design is measured before it is built into the
// verify path.  Values are arbitrary field elements (the code has no data-dependent
// branches), results are written out only to keep the work live.
//
//   ml_simt_w1 / _w2 : one optimal-ate Miller loop per lane (bls/pairing.hpp
//                      miller_loop: f in registers, no squaring shared between pairs),
//                      register budget for 1 or 2 wavefronts per SIMD
//   fpm_d28          : a dependent chain of 28-bit-digit Montgomery products per lane
//   glv_g1           : [s] P on G1 by jac_mul_glv with the window table in LDS (k_pset's
//                      second wavefront), one point per lane
#define BLS_FP_D28 1
#include <string>

#include "../launchers.hpp"
#include "bls/pairing.hpp"

using namespace bls;

namespace {

__device__ Fp probe_fp(uint32_t lane, uint32_t k) {
  Fp r;
  uint32_t s = lane * 0x9e3779b9u + k * 0x85ebca6bu + 1u;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    r.l[i] = s;
  }
  r.l[11] &= 0x0fffffffu;  // < p
  return r;
}

__device__ void probe_ml(Fp12* out, uint32_t n) {
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  G1A P;
  P.x = probe_fp(i, 0);
  P.y = probe_fp(i, 1);
  P.inf = false;
  G2A Q;
  Q.x = Fp2{probe_fp(i, 2), probe_fp(i, 3)};
  Q.y = Fp2{probe_fp(i, 4), probe_fp(i, 5)};
  Q.inf = false;
  out[i] = miller_loop(g1_eval_from_aff(P), Q);
}

}  // namespace

__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(1))) void k_probe_ml_w1(Fp12* out,
                                                                                                     uint32_t n) {
  probe_ml(out, n);
}

__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(2))) void k_probe_ml_w2(Fp12* out,
                                                                                                     uint32_t n) {
  probe_ml(out, n);
}

__global__ __launch_bounds__(BLS_BLOCK) void k_probe_fpm_d28(Fp* io, uint32_t n) {
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  Fp a = probe_fp(i, 0), b = probe_fp(i, 1);
  for (int k = 0; k < 256; ++k) a = fp_mul_lazy(a, b);
  io[i] = a;
}

__global__ __launch_bounds__(BLS_BLOCK) void k_probe_glv_g1(G1J* out, uint32_t n) {
  __shared__ G1J tab[4][15];
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n || threadIdx.x >= 4) return;
  const G1J p = jac_from_aff(g1_generator());
  uint32_t a, b;
  glv_split(0x9e3779b97f4a7c15ull * (i + 1), a, b);
  out[i] = jac_mul_glv<Fp>(p, a, b, tab[threadIdx.x]);
}

// bytes of output per lane for probe `name`, or 0 if unknown
size_t kernel_probe_out_bytes(const char* name) {
  const std::string s(name);
  if (s == "ml_simt_w1" || s == "ml_simt_w2") return sizeof(Fp12);
  if (s == "fpm_d28") return sizeof(Fp);
  if (s == "glv_g1") return sizeof(G1J);
  return 0;
}

hipError_t launch_kernel_probe(const char* name, void* out, uint32_t lanes, hipStream_t st) {
  const std::string s(name);
  const unsigned grid = bls_grid_for(lanes);
  if (s == "ml_simt_w1") k_probe_ml_w1<<<grid, BLS_BLOCK, 0, st>>>((Fp12*)out, lanes);
  else if (s == "ml_simt_w2") k_probe_ml_w2<<<grid, BLS_BLOCK, 0, st>>>((Fp12*)out, lanes);
  else if (s == "glv_g1") k_probe_glv_g1<<<grid, BLS_BLOCK, 0, st>>>((G1J*)out, lanes);
  else if (s == "fpm_d28") k_probe_fpm_d28<<<grid, BLS_BLOCK, 0, st>>>((Fp*)out, lanes);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
