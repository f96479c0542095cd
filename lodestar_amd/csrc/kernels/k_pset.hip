// Per-set cooperative kernel: one 64-lane wavefront per signature set runs the
// "pset" programs of tools/gen_pset.py (interpreter: bls/coop.hpp):
//
//   P = iso(q0) + iso(q1)                               pset_prep
//   for the 64 bits of r (and the fixed bits of |x|):   pset_dbl_r / pset_dbl_all,
//       A = [|x|]P, C = [|x|]sig, D = [r + 2^64](sig, pk), E = [2^64](sig, pk)
//                                                       pset_add_x / _r / _xr
//   H = clear_cofactor(P), r sig = D1 - E1, r pk = D2 - E2, psi(sig) ?= [x]sig
//                                                       pset_phase2
//   affine H and r sig with one lane-0 inversion        pset_norm2, pset_affine2
//   f_i = ML(r pk, H) * ML(-g1, r sig)                  pset_ml2
//
// Reference semantics: Signature.fromBytes(.., validate=true) (maybeBatch.ts:23,36)
// for the subgroup test, hash_to_G2 + the random-scalar pairing product of
// verifyMultipleSignatures ([ext] blst) for f_i.  A zero-checked exceptional
// addition, an infinity signature or a flag from k_pre sends the set to k_exact
// (pipeline.hpp stage_exact_set; kept out of this kernel so its registers and
// stack do not lower this kernel's occupancy).  Flagged sets are counted; the host
// launches k_exact (and redoes status + chunks) only when the count is non-zero.
#include "../launchers.hpp"

using namespace bls;

typedef CoopLds PsetShared;

// frame registers (tools/gen_pset.py)
enum : int { PS_Q0 = 0, PS_SIG = 8, PS_PK = 12, PS_INV_IN = 74, PS_INV_OUT = 75, PS_DIFF = 76, PS_F = 80 };

#define PS_X_ABS 0xD201000000010000ull

__device__ __forceinline__ void pset_store_one(Fp12* dst) {
  Fp* d = reinterpret_cast<Fp*>(dst);
  if (threadIdx.x < 12) d[threadIdx.x] = threadIdx.x == 0 ? c_one() : fp_zero();
}

// hand the set to the exact path (lane 0)
__device__ __forceinline__ void pset_flag(const PipeBufs& b, uint32_t i) {
  b.set_flag[i] = 1u;
  atomicAdd(b.flag_count, 1u);
}

__global__ __launch_bounds__(COOP_LANES) void k_pset(PipeBufs b, CoopEnv env) {
  __shared__ PsetShared sh;
  const uint32_t i = blockIdx.x;
  const int lane = threadIdx.x;
  if (b.pk_status[i] != BLS_OK || b.sig_status[i] != BLS_OK || jac_is_inf(b.pk[i])) {
    pset_store_one(&b.f[i]);  // the request errors on its status; f_i is unused
    return;
  }
  if (b.sig[i].inf || b.set_flag[i]) {
    if (lane == 0) pset_flag(b, i);
    return;
  }
  coop_stage_consts(env, sh.cbank);
  if (lane < 8) lds_store_fp(sh.frame, PS_Q0 + lane, b.q[8ull * i + lane]);
  if (lane >= 8 && lane < 12) lds_store_fp(sh.frame, PS_SIG + lane - 8, reinterpret_cast<const Fp*>(&b.sig[i])[lane - 8]);
  if (lane >= 12 && lane < 15) lds_store_fp(sh.frame, PS_PK + lane - 12, reinterpret_cast<const Fp*>(&b.pk[i])[lane - 12]);
  if (lane == 0) sh.flag = 0;
  __syncthreads();
  const uint64_t r = set_scalar(b.seed, b.scalar_base + i);

  coop_run(env, env.pset_prep, sh.frame, sh.cbank, &sh.flag);
  coop_run(env, env.pset_dbl_r, sh.frame, sh.cbank, &sh.flag);
  if ((r >> 63) & 1ull) coop_run(env, env.pset_add_r, sh.frame, sh.cbank, &sh.flag);
  for (int k = 62; k >= 0; --k) {
    coop_run(env, env.pset_dbl_all, sh.frame, sh.cbank, &sh.flag);
    const bool xb = (PS_X_ABS >> k) & 1ull, rb = (r >> k) & 1ull;
    if (xb && rb) coop_run(env, env.pset_add_xr, sh.frame, sh.cbank, &sh.flag);
    else if (xb) coop_run(env, env.pset_add_x, sh.frame, sh.cbank, &sh.flag);
    else if (rb) coop_run(env, env.pset_add_r, sh.frame, sh.cbank, &sh.flag);
  }
  coop_run(env, env.pset_phase2, sh.frame, sh.cbank, &sh.flag);
  if (sh.flag) {
    if (lane == 0) pset_flag(b, i);
    return;
  }
  if (!coop_is_zero(sh.frame, PS_DIFF, 4)) {  // psi(sig) != [x] sig: not in G2
    if (lane == 0) b.sig_status[i] = BLS_POINT_NOT_IN_GROUP;
    pset_store_one(&b.f[i]);
    return;
  }
  coop_run(env, env.pset_norm2, sh.frame, sh.cbank, &sh.flag);
  if (sh.flag) {
    if (lane == 0) pset_flag(b, i);
    return;
  }
  coop_invert(sh.frame, PS_INV_IN, PS_INV_OUT);
  coop_run(env, env.pset_affine2, sh.frame, sh.cbank, &sh.flag);
  coop_run(env, env.pset_ml2, sh.frame, sh.cbank, &sh.flag);
  if (lane < 12) reinterpret_cast<Fp*>(&b.f[i])[lane] = coop_get(sh.frame, PS_F + lane);
}

hipError_t launch_k_pset(const PipeBufs& b, const CoopEnv& env, hipStream_t s) {
  k_pset<<<b.n_sets, COOP_LANES, 0, s>>>(b, env);
  return hipGetLastError();
}
