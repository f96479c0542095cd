// Cooperative per-set stages (one 64-lane wavefront per signature set; programs
// from tools/gen_coop.py "set" frame, interpreter in bls/coop.hpp):
//   k_miller_coop  f_i = ML(r_i pk_i, H(m_i)), the G1 point in Jacobian form
#include "../launchers.hpp"

using namespace bls;

struct SetShared {
  Fp frame[COOP_FRAME];
  Fp cbank[COOP_MAX_CONSTS];
  uint32_t flag;
};

enum : int { SET_Q = 0, SET_P = 4, SET_F = 8 };

__device__ __forceinline__ void store_fp12_one(Fp12* dst) {
  Fp* d = reinterpret_cast<Fp*>(dst);
  if (threadIdx.x < 12) d[threadIdx.x] = threadIdx.x == 0 ? c_one() : fp_zero();
}

__global__ __launch_bounds__(COOP_LANES) void k_miller_coop(PipeBufs b, CoopEnv env) {
  __shared__ SetShared sh;
  const uint32_t i = blockIdx.x;
  const bool live = b.pk_status[i] == BLS_OK && b.sig_status[i] == BLS_OK && !fp_is_zero(b.rpk[i].z) && !b.H[i].inf;
  if (!live) {
    store_fp12_one(&b.f[i]);
    return;
  }
  coop_stage_consts(env, sh.cbank);
  if (threadIdx.x < 4) lds_store_fp(sh.frame, SET_Q + threadIdx.x, reinterpret_cast<const Fp*>(&b.H[i])[threadIdx.x]);
  if (threadIdx.x >= 4 && threadIdx.x < 7)
    lds_store_fp(sh.frame, SET_P + threadIdx.x - 4, reinterpret_cast<const Fp*>(&b.rpk[i])[threadIdx.x - 4]);
  if (threadIdx.x == 0) sh.flag = 0;
  __syncthreads();
  coop_run(env, env.set_ml, sh.frame, sh.cbank, &sh.flag);
  if (threadIdx.x < 12) reinterpret_cast<Fp*>(&b.f[i])[threadIdx.x] = lds_load_fp(sh.frame, SET_F + threadIdx.x);
}

hipError_t launch_k_miller_coop(const PipeBufs& b, const CoopEnv& env, hipStream_t s) {
  k_miller_coop<<<b.n_sets, COOP_LANES, 0, s>>>(b, env);
  return hipGetLastError();
}
