// Per-set scalar chains of the aggregated-signature path, one lane per set (SIMT):
// everything of a set's work except its Miller loop.
//
//   in_group = psi(sig) == [x] sig         (Scott's G2 test: Signature.fromBytes(.., true),
//                                           maybeBatch.ts:23,36)
//   P  = iso(q0) + iso(q1)                 (Jacobian isogeny, no inversion)
//   H  = clear_cofactor(P), affine         (RFC 9380 Budroni-Pintore, one inversion)
//   RP = [r] pk,  RS = [r] sig             (the 64-bit batch scalar of
//                                           verifyMultipleSignatures, [ext] blst)
//
// The batch equation prod e(r_i pk_i, H_i) * e(-g1, sum r_i sig_i) == 1 is then
// evaluated as the reference's blst does it: one Miller loop per set for (RP, H)
// (k_mlq / k_mlf, kernels/k_mlq.hip) and ONE per pass for (-g1, sum RS) (the merged
// signature sum: k_msm's Pippenger sum, or k_gsum's group sums of the RS with k_vset
// turning a sum into a virtual set).
//
// These are narrow, strictly sequential double-and-add chains (about 6k Fp products
// per set: 3 G2 chains over |x|, one over r, one G1 chain over r): one lane per set
// keeps all 64 lanes busy, where the cooperative interpreter filled 20..50 of 64
// lanes per step with them.  The point formulas are curve.hpp's complete ones
// (infinity and doubling branches), so no addition needs the exact path; the set
// goes to k_exact only for an infinity signature, an SSWU input k_pre flagged,
// H = O, or [r] pk = O (a pubkey outside G1).
//
// Output per live set (b.chain, CH_* layout); b.chain_live[i] = 1 (k_chain_done).  A
// set whose request errors (decode status, infinity pubkey) or whose signature is
// outside G2 gets f_i = 1 and is not live (not summed, no Miller loop).
// The 28-bit-digit product (bls/field.hpp) is called out of line; inlined into these
// chains the kernel needs 4,544 B of scratch per lane, a reservation of 568 MiB per
// queue that took the runtime past its scratch grant with the bench's queues (DESIGN.md
// §3, profiles/r03_chain_inl28_resources.txt) -- the round-2 "never finished".
#define BLS_FP_D28 1
#include "../launchers.hpp"

using namespace bls;

namespace {

// out-of-line isogeny (bls/hash_to_curve.hpp iso_map_jac), called twice per set
__device__ __noinline__ void iso_jac_nl(G2J* out, const Fp* q) { *out = iso_map_jac(Fp2{q[0], q[1]}, Fp2{q[2], q[3]}); }

// One out-of-line copy of each chain (the two [x] chains of H and the subgroup test on
// affine bases, RS on the affine signature, RP on G1): the double-and-add body is large,
// so the kernel keeps a single instance of it.
// affine base: mixed additions
__device__ __noinline__ void g2_mul_aff(G2J* out, const G2A* in, uint64_t k) { *out = aff_mul_u64(*in, k); }
// [r] sig and [r] pk for the per-set batch scalar r: GLV/GLS (curve.hpp jac_mul_glv):
// the set's scalar is a + b mu with a, b its two 32-bit halves and mu = -x^2, applied as
// [a]P + [b]endo(P) through a joint 2-bit window -- 33 doublings instead of 63 (G1:
// sigma(x, y) = (beta x, y); G2: -psi^2).  The window's table of points lives in the
// call's workspace (PipeBufs::rtab2 / rtab1), not in private memory.  (Double-and-add
// and a fixed 4-bit window over the 64-bit scalar measured slower,
// profiles/r02c_ab_chain_window.json.)
__device__ __noinline__ void g2_mul_r(G2J* out, const G2A* in, uint64_t k, G2J* T) {
  uint32_t a, b;
  glv_split(k, a, b);
  *out = in->inf ? jac_infinity<Fp2>() : jac_mul_glv<Fp2>(jac_from_aff(*in), a, b, T);
}
__device__ __noinline__ void g1_mul_r(G1J* out, const G1J* in, uint64_t k, G1J* T) {
  uint32_t a, b;
  glv_split(k, a, b);
  *out = jac_mul_glv<Fp>(*in, a, b, T);
}
// out-of-line general addition for the handful of additions outside the chains
__device__ __noinline__ void g2_add(G2J* out, const G2J* a, const G2J* b) { *out = jac_add(*a, *b); }

// affine form of a Jacobian G2 point by one Fp inversion of N(Z) (binary GCD)
__device__ __noinline__ void g2_to_aff(G2A* out, const G2J* in) {
  if (jac_is_inf(*in)) {
    out->x = fp2_zero();
    out->y = fp2_zero();
    out->inf = true;
    return;
  }
  const Fp ni = fp_inv_gcd(fp_add(fp_sqr(in->z.c0), fp_sqr(in->z.c1)));
  const Fp2 zi = Fp2{fp_mul(in->z.c0, ni), fp_neg(fp_mul(in->z.c1, ni))};
  const Fp2 zi2 = fp2_sqr(zi);
  out->x = fp2_mul(in->x, zi2);
  out->y = fp2_mul(in->y, fp2_mul(zi2, zi));
  out->inf = false;
}

// [x]P = -[|x|]P over the affine form of P: the chain's five additions are mixed
// (madd-2007-bl, 29 Fp products instead of add-2007-bl's 43) for one inversion
__device__ __noinline__ void g2_mul_x_aff(G2J* out, const G2J* p) {
  G2A a;
  g2_to_aff(&a, p);
  g2_mul_aff(out, &a, (uint64_t)BLS_X_ABS);
  out->y = fp2_neg(out->y);
}

__device__ void store_one(Fp12* f) {
  Fp* d = reinterpret_cast<Fp*>(f);
  d[0] = c_one();
#pragma unroll
  for (int k = 1; k < 12; ++k) d[k] = fp_zero();
}

__device__ void flag_exact(const PipeBufs& b, uint32_t i) {
  b.set_flag[i] = 1u;
  atomicAdd(b.flag_count, 1u);
}

}  // namespace

// the set needs no chains: its request errors on its status (f_i = 1), or the exact
// path takes it (infinity signature, SSWU flag from k_pre)
__device__ bool chain_skip(const PipeBufs& b, uint32_t i) {
  return b.pk_status[i] != BLS_OK || b.sig_status[i] != BLS_OK || jac_is_inf(b.pk[i]) || b.sig[i].inf ||
         b.set_flag[i];
}

// The four roles, each out of line: the kernel's scratch is then the largest role's
// frame, not the kernel frame holding role 0's points plus the deepest callee (the
// runtime reserves scratch per queue for a full device of wavefronts,
// lodestar_amd/build.py SCRATCH_BUDGET).
// The role functions take the buffers they use as plain pointers: a `const PipeBufs&`
// made the kernel copy its whole argument block into private memory (a 480-byte frame
// under every role).
__device__ __noinline__ void chain_role_h(Fp* chain, const Fp* qs, uint8_t* chain_st, uint32_t i) {
  Fp* o = chain + (size_t)CHAIN_WORDS * i;
  // H = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P), P = iso(q0) + iso(q1) (RFC 9380
  // G.3), regrouped so one point stays live across each [x] chain and four additions
  // remain instead of five:
  //   s = [x]P + psi(P),   u = psi^2(2P) - (s + P),   H = [x]s + u
  // (the same group element by the complete formulas, so the same affine H)
  // Three point slots in private memory, reused in place (the out-of-line helpers take
  // pointers; a fresh temporary per step made a 2.6 KB frame)
  const Fp* q = qs + 8ull * i;
  G2J A, B, C;
  iso_jac_nl(&A, q);
  iso_jac_nl(&B, q + 4);
  g2_add(&A, &A, &B);             // A = P
  g2_mul_x_aff(&B, &A);           // B = [x]P
  C = g2_psi(A);
  g2_add(&B, &B, &C);             // B = s
  C = g2_psi(g2_psi(jac_dbl(A)));
  g2_add(&A, &B, &A);
  A.y = fp2_neg(A.y);
  g2_add(&C, &C, &A);             // C = u
  g2_mul_x_aff(&A, &B);           // A = [x]s
  g2_add(&A, &A, &C);             // A = H
  chain_st[4 * i + 0] = jac_is_inf(A) ? 1 : 0;
  if (jac_is_inf(A)) return;
  // HQ = affine H: one Fp inversion of N(Z) (inline here: through g2_to_aff the frame
  // grows by the affine point's slot)
  const Fp ni = fp_inv_gcd(fp_add(fp_sqr(A.z.c0), fp_sqr(A.z.c1)));
  const Fp2 zi = Fp2{fp_mul(A.z.c0, ni), fp_neg(fp_mul(A.z.c1, ni))};
  const Fp2 zi2 = fp2_sqr(zi);
  const Fp2 hx = fp2_mul(A.x, zi2);
  const Fp2 hy = fp2_mul(A.y, fp2_mul(zi2, zi));
  o[CH_HQ + 0] = hx.c0;
  o[CH_HQ + 1] = hx.c1;
  o[CH_HQ + 2] = hy.c0;
  o[CH_HQ + 3] = hy.c1;
}

__device__ __noinline__ void chain_role_sub(const G2A* sigs, uint8_t* chain_st, uint32_t i) {
  const G2A sig = sigs[i];
  G2J xs;
  g2_mul_aff(&xs, &sig, (uint64_t)BLS_X_ABS);
  chain_st[4 * i + 1] = jac_eq(g2_psi(jac_from_aff(sig)), jac_neg(xs)) ? 0 : 1;
}

__device__ __noinline__ void chain_role_rs(Fp* chain, const G2A* sigs, const uint32_t* seed, uint32_t scalar_base,
                                           G2J* rtab2, uint32_t i) {
  Fp* o = chain + (size_t)CHAIN_WORDS * i;
  const G2A sig = sigs[i];
  G2J RS;
  g2_mul_r(&RS, &sig, set_scalar(seed, scalar_base + i), rtab2 + 15ull * i);
  o[CH_RS + 0] = RS.x.c0;
  o[CH_RS + 1] = RS.x.c1;
  o[CH_RS + 2] = RS.y.c0;
  o[CH_RS + 3] = RS.y.c1;
  o[CH_RS + 4] = RS.z.c0;
  o[CH_RS + 5] = RS.z.c1;
}

__device__ __noinline__ void chain_role_rp(Fp* chain, const G1J* pks, uint8_t* chain_st, const uint32_t* seed,
                                           uint32_t scalar_base, G1J* rtab1, uint32_t i) {
  Fp* o = chain + (size_t)CHAIN_WORDS * i;
  G1J RP;
  const G1J pk = pks[i];
  g1_mul_r(&RP, &pk, set_scalar(seed, scalar_base + i), rtab1 + 15ull * i);
  chain_st[4 * i + 3] = jac_is_inf(RP) ? 1 : 0;
  if (jac_is_inf(RP)) return;
  o[CH_RP + 0] = RP.x;
  o[CH_RP + 1] = RP.y;
  o[CH_RP + 2] = RP.z;
}

// Four roles per set, one wavefront per (role, 64 sets), so a call of n sets runs
// 4 n / 64 wavefronts and its latency is the longest chain, not their sum (one kernel
// per role, each with its own register budget, measured 5 % slower at 14 and 16
// contexts x 8 calls: the four launches serialise on the context's stream,
// profiles/r03_ab_chain_roles.json):
//   role 0  H = clear_cofactor(iso(q0) + iso(q1)) -> HQ (affine)   ~2.9k Fp products,
//           once per distinct signing root
//   role 1  psi(sig) == [x] sig                                     ~1.2k
//   role 2  RS = [r] sig                                            ~1.9k
//   role 3  RP = [r] pk                                             ~1.0k
// Results that decide the set's fate go to b.chain_st[4 i + role] (k_chain_done
// reads them; every role that runs writes its byte, so no clearing is needed).
// At most 256 VGPRs, so two wavefronts share a SIMD: cfg2 +1.2 % over one 394-VGPR
// wavefront per SIMD (profiles/r02b_ab_chain_occ2.json); one or three per SIMD were
// slower (profiles/r02c_ab_chain_occ.json).
#define BLS_CHAIN_ATTR __attribute__((amdgpu_waves_per_eu(2)))
__global__ __launch_bounds__(BLS_BLOCK) BLS_CHAIN_ATTR void k_chain(PipeBufs b, uint32_t blocks_per_role,
                                                                   uint32_t roles) {
  // the (blockIdx / blocks_per_role)-th role present in the mask
  uint32_t role = 0, nth = blockIdx.x / blocks_per_role;
  for (uint32_t m = roles;; m &= m - 1) {
    if (nth-- == 0) {
      role = (uint32_t)__builtin_ctz(m);
      break;
    }
  }
  const uint32_t i = (blockIdx.x % blocks_per_role) * BLS_BLOCK + threadIdx.x;
  if (i >= b.n_sets) return;
  // H(m) once per distinct signing root: only the root's first set
  // (plan_msg_dedup) runs role 0, whatever its own pubkey / signature status, unless
  // its SSWU points went to the exact path; k_chain_done shares the result
  if (role == 0 ? ((b.msg_rep && b.msg_rep[i] != i) || b.set_flag[i]) : chain_skip(b, i)) return;
  if (role == 0) chain_role_h(b.chain, b.q, b.chain_st, i);
  else if (role == 1) chain_role_sub(b.sig, b.chain_st, i);
  else if (role == 2) chain_role_rs(b.chain, b.sig, b.seed, b.scalar_base, b.rtab2, i);
  else chain_role_rp(b.chain, b.pk, b.chain_st, b.seed, b.scalar_base, b.rtab1, i);
}

// One lane per set after the four roles: the set's fate.
__global__ __launch_bounds__(BLS_BLOCK) void k_chain_done(PipeBufs b) {
  BLS_TAIL_PRIO();
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= b.n_sets) return;
  b.chain_live[i] = 0u;
  if (b.pk_status[i] != BLS_OK || b.sig_status[i] != BLS_OK || jac_is_inf(b.pk[i])) {
    store_one(&b.f[i]);  // the request errors on its status; f_i is unused
    return;
  }
  if (b.sig[i].inf || b.set_flag[i]) {
    flag_exact(b, i);
    return;
  }
  const uint8_t* st = b.chain_st + 4 * i;
  if (st[1]) {  // psi(sig) != [x] sig: Signature.fromBytes(.., validate) throws
    b.sig_status[i] = BLS_POINT_NOT_IN_GROUP;
    store_one(&b.f[i]);
    return;
  }
  const uint32_t rep = b.msg_rep ? b.msg_rep[i] : i;  // the set that computed this root's H
  if (b.chain_st[4 * rep + 0] || st[3]) {  // H = O or [r] pk = O: the exact path's complete formulas decide
    flag_exact(b, i);
    return;
  }
  if (rep != i) {
    const Fp* src = b.chain + (size_t)CHAIN_WORDS * rep + CH_HQ;
    Fp* dst = b.chain + (size_t)CHAIN_WORDS * i + CH_HQ;
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = src[k];
  }
  if (b.set_unit && b.set_unit[i] != UNIT_NONE) store_one(&b.f[i]);  // paired in its unit
  b.chain_live[i] = 1u;
}

hipError_t launch_k_chain(const PipeBufs& b, hipStream_t s, uint32_t roles) {
  const uint32_t nb = bls_grid_for(b.n_sets);
  roles &= 0xFu;
  if (roles == 0) return hipSuccess;
  k_chain<<<(uint32_t)__builtin_popcount(roles) * nb, BLS_BLOCK, 0, s>>>(b, nb, roles);
  if (roles != 0x4u) k_chain_done<<<nb, BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
