// Per-set cooperative kernel: one 64-lane wavefront per signature set runs the "pset"
// programs of tools/gen_pset.py (interpreter: bls/coop.hpp):
//
//   P = iso(q0) + iso(q1)                               pset_prep
//   A = [|x|]P, C = [|x|]sig (fixed bits of |x|)        pset_xchain (pset_dbl_all / pset_add_x
//                                                       in the order of |x|'s bits)
//   H = clear_cofactor(P), psi(sig) ?= [x]sig           pset_phase2
//   affine H with one lane-0 inversion                  pset_norm2, pset_affine2
//   f_i = ML(RP, H) * ML(-RG, sig)                      pset_ml2
//
// RG = [s] g1 and RP = [s] pk for the set's batch scalar s come from k_pre's extra lanes
// (GLV, kernels/k_pre.hip pre_rpts), computed beside the SSWU maps: the r chains used to
// run here as interpreter programs beside the |x| chains (a 64-bit double-and-add, ~290
// more steps on the set's critical path; then a second wavefront of this kernel, which
// slowed the first by 0.35 ms, profiles/r04_ab_pset_rpoints.json).
//
// Reference semantics: Signature.fromBytes(.., validate=true) (maybeBatch.ts:23,36)
// for the subgroup test, hash_to_G2 + the random-scalar pairing product of
// verifyMultipleSignatures ([ext] blst) for f_i.  A zero-checked exceptional
// addition, an infinity signature, RP at infinity (a public key of small order, flagged
// by k_pre) or another flag from k_pre sends the set to k_exact (pipeline.hpp
// stage_exact_set; kept out of this kernel so its registers and stack do not lower this
// kernel's occupancy).  Flagged sets are counted; the host launches k_exact (and redoes
// status + chunks) only when the count is non-zero.
#define BLS_FP_D28 1  // 28-bit-digit Montgomery product (bls/field.hpp)
#include "../launchers.hpp"

using namespace bls;

typedef CoopLds PsetShared;

// frame registers (tools/gen_pset.py)
enum : int {
  PS_Q0 = 0,
  PS_SIG = 8,
  PS_PK = 12,
  PS_RG = 57,
  PS_RP = 63,
  PS_INV_IN = 74,
  PS_INV_OUT = 75,
  PS_DIFF = 76,
  PS_F = 80
};

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

// Two wavefronts per set: wavefront 0 runs every program up to the Miller loop (their
// steps fit one wavefront with each product and combination on a lane pair, coop.hpp
// coop_step); both run the Miller loop, whose steps carry ~48 products -- 96 lanes as
// pairs (pset_ml2_w2, tools/gen_coop.py).  Every branch between the block barriers below
// reads block-uniform values (the set's status in global memory, the LDS flag and frame
// after a barrier), so both wavefronts take it.
#define PSET_WAVES 2
__global__ __launch_bounds__(PSET_WAVES * COOP_LANES) void k_pset(PipeBufs b, const CoopEnv* __restrict__ envp) {
  const CoopEnv& env = *envp;
  __shared__ PsetShared sh;
  const uint32_t i = blockIdx.x;
  const int lane = threadIdx.x;
  const bool w0 = lane < COOP_LANES;
  if (b.pk_status[i] != BLS_OK || b.sig_status[i] != BLS_OK || jac_is_inf(b.pk[i])) {
    pset_store_one(&b.f[i]);  // the request errors on its status; f_i is unused
    return;
  }
  if (b.sig[i].inf || b.set_flag[i]) {
    if (lane == 0) pset_flag(b, i);
    return;
  }
  coop_stage_consts(env, sh.cbank);
  const Fp* rp = reinterpret_cast<const Fp*>(b.rpts + 2ull * i);  // RP (x, y, z), RG (x, y, z)
  if (lane < 8) lds_store_fp(sh.frame, PS_Q0 + lane, b.q[8ull * i + lane]);
  if (lane >= 8 && lane < 12) lds_store_fp(sh.frame, PS_SIG + lane - 8, reinterpret_cast<const Fp*>(&b.sig[i])[lane - 8]);
  if (lane >= 12 && lane < 15) lds_store_fp(sh.frame, PS_PK + lane - 12, reinterpret_cast<const Fp*>(&b.pk[i])[lane - 12]);
  if (lane >= 15 && lane < 18) lds_store_fp(sh.frame, PS_RP + lane - 15, rp[lane - 15]);
  if (lane >= 18 && lane < 21) lds_store_fp(sh.frame, PS_RG + lane - 18, rp[3 + lane - 18]);
  if (lane == 0) sh.flag = 0;
  __syncthreads();

  if (w0) {
    coop_run(env, env.pset_prep, sh.frame, sh.cbank, &sh.flag);
    coop_run(env, env.pset_xchain, sh.frame, sh.cbank, &sh.flag);  // 63 doublings, 5 additions
    coop_run(env, env.pset_phase2, sh.frame, sh.cbank, &sh.flag);
  }
  __syncthreads();
  if (sh.flag) {
    if (lane == 0) pset_flag(b, i);
    return;
  }
  if (!coop_is_zero(sh.frame, PS_DIFF, 4)) {  // psi(sig) != [x] sig: not in G2
    if (lane == 0) b.sig_status[i] = BLS_POINT_NOT_IN_GROUP;
    pset_store_one(&b.f[i]);
    return;
  }
  if (w0) coop_run(env, env.pset_norm2, sh.frame, sh.cbank, &sh.flag);
  __syncthreads();
  if (sh.flag) {
    if (lane == 0) pset_flag(b, i);
    return;
  }
  if (w0) {
    coop_invert(sh.frame, PS_INV_IN, PS_INV_OUT);
    coop_run(env, env.pset_affine2, sh.frame, sh.cbank, &sh.flag);
  }
  __syncthreads();
  coop_run2_t(env, env.pset_ml2_w2, sh.frame, &sh.flag);
  if (lane < 12) reinterpret_cast<Fp*>(&b.f[i])[lane] = coop_get(sh.frame, PS_F + lane);
}

// S sets per wavefront (tools/gen_pset.py build_pset(S): set s at frame offset 92 s,
// its zero-checks on flag bit s).  The same programs as k_pset scheduled jointly: the
// narrow chains of one set leave most lanes idle, so further sets ride along at
// almost no extra steps (the |x| chains and phase 2 unchanged; Miller loop ~690 steps for
// 2 sets, ~920 for 3, vs 486 for 1); RG and RP from k_pre as in k_pset.  A set that needs no programs (error status,
// flagged) borrows the inputs of the first live set so every part of the frame holds
// well-formed points; its results are dropped.  Controller decisions (program
// choice, early exits) are wave-uniform.
#define PSN_SLOTS 92

template <int S, int FRAME_N>
__global__ __launch_bounds__(COOP_LANES) void k_psetn(PipeBufs b, const CoopEnv* __restrict__ envp) {
  const CoopEnv& env = *envp;
  __shared__ CoopLdsN<FRAME_N> sh;
  const CoopPsetN& pg = env.packed[S - 2];
  const int lane = threadIdx.x;
  const uint32_t i0 = (uint32_t)S * blockIdx.x;
  bool live[S];
  int first_live = -1;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint32_t i = i0 + s;
    live[s] = false;
    if (i >= b.n_sets) continue;
    if (b.pk_status[i] != BLS_OK || b.sig_status[i] != BLS_OK || jac_is_inf(b.pk[i])) {
      pset_store_one(&b.f[i]);
    } else if (b.sig[i].inf || b.set_flag[i]) {
      if (lane == 0) pset_flag(b, i);
    } else {
      live[s] = true;
      if (first_live < 0) first_live = s;
    }
  }
  if (first_live < 0) return;
  uint32_t src[S];
#pragma unroll
  for (int s = 0; s < S; ++s) src[s] = i0 + (live[s] ? s : first_live);
  coop_stage_consts(env, sh.cbank);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint32_t i = src[s], o = PSN_SLOTS * s;
    const Fp* rp = reinterpret_cast<const Fp*>(b.rpts + 2ull * i);  // RP (x, y, z), RG (x, y, z)
    if (lane < 8) lds_store_fp(sh.frame, o + PS_Q0 + lane, b.q[8ull * i + lane]);
    if (lane >= 8 && lane < 12)
      lds_store_fp(sh.frame, o + PS_SIG + lane - 8, reinterpret_cast<const Fp*>(&b.sig[i])[lane - 8]);
    if (lane >= 12 && lane < 15)
      lds_store_fp(sh.frame, o + PS_PK + lane - 12, reinterpret_cast<const Fp*>(&b.pk[i])[lane - 12]);
    if (lane >= 15 && lane < 18) lds_store_fp(sh.frame, o + PS_RP + lane - 15, rp[lane - 15]);
    if (lane >= 18 && lane < 21) lds_store_fp(sh.frame, o + PS_RG + lane - 18, rp[3 + lane - 18]);
  }
  if (lane == 0) sh.flag = 0;
  __syncthreads();

  coop_run(env, pg.prep, sh.frame, sh.cbank, &sh.flag);
  for (int k = 62; k >= 0; --k) {
    coop_run(env, pg.dbl_all, sh.frame, sh.cbank, &sh.flag);
    if ((PS_X_ABS >> k) & 1ull) coop_run(env, pg.add_x, sh.frame, sh.cbank, &sh.flag);
  }
  coop_run(env, pg.phase2, sh.frame, sh.cbank, &sh.flag);
  bool run[S];
  bool any = false;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    run[s] = live[s];
    if (!run[s]) continue;
    const uint32_t i = i0 + s;
    if ((sh.flag >> s) & 1u) {
      if (lane == 0) pset_flag(b, i);
      run[s] = false;
    } else if (!coop_is_zero(sh.frame, PSN_SLOTS * s + PS_DIFF, 4)) {  // psi(sig) != [x] sig: not in G2
      if (lane == 0) b.sig_status[i] = BLS_POINT_NOT_IN_GROUP;
      pset_store_one(&b.f[i]);
      run[s] = false;
    }
    any = any || run[s];
  }
  if (!any) return;
  coop_run(env, pg.norm2, sh.frame, sh.cbank, &sh.flag);
  any = false;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (run[s] && ((sh.flag >> s) & 1u)) {
      if (lane == 0) pset_flag(b, i0 + s);
      run[s] = false;
    }
    any = any || run[s];
  }
  if (!any) return;
  // all S inversions at once (lanes 0..S-1; fp_inv_gcd(0) = 0 for a dropped part)
  if (lane < S) {
    const int o = PSN_SLOTS * lane;
    lds_store_fp(sh.frame, o + PS_INV_OUT, fp_inv_gcd(fp_canon3(lds_load_fp(sh.frame, o + PS_INV_IN))));
  }
  __syncthreads();
  coop_run(env, pg.affine2, sh.frame, sh.cbank, &sh.flag);
  coop_run(env, pg.ml2, sh.frame, sh.cbank, &sh.flag);
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (run[s] && lane < 12)
      reinterpret_cast<Fp*>(&b.f[i0 + s])[lane] = coop_get(sh.frame, PSN_SLOTS * s + PS_F + lane);
}

// Single-pair Miller loops of the aggregated-signature path (after k_chain.hip and
// k_gsum.hip's k_vset): S sets per wavefront, f_i = ML(RP_i, HQ_i) for the sets in
// [first, first + count) that are live (real sets: RP = [r] pk, HQ = H(m); a group's
// virtual set: RP = -g1, HQ = sum r sig).  Frame per packed set s (tools/gen_pset.py
// build_ml1, ML1_SLOTS = 19): RP at 19 s + 0..2, HQ at 19 s + 3..6, F at 19 s + 7..18.
// A part of the wave with no live set borrows the first live set's inputs.
enum : int { ML1_SLOTS = 19, ML1_RP = 0, ML1_HQ = 3, ML1_F = 7 };

// S items starting at i0 on an LDS frame: the single-pair loops (ml1_S, constants
// staged at slot cb, the frame size that program was scheduled for).  The body of
// k_mln<S>.
template <int S>
__device__ __forceinline__ void mln_items(const PipeBufs& b, const CoopEnv& env, Fp* frame, uint32_t* flag,
                                          int cb, uint32_t i0, uint32_t end, uint32_t units_paired) {
  const CoopProg& ml = S == 1 ? env.ml1_1 : env.ml1_2;
  const int lane = threadIdx.x;
  bool live[S];
  int first_live = -1;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint32_t i = i0 + s;
    // a set paired inside its Miller-loop unit has f_i = 1 here (units_paired: the
    // first pass), but runs its own loop when its request is verified alone
    live[s] = i < end && b.chain_live[i] &&
              !(units_paired && b.set_unit && i < b.n_sets && b.set_unit[i] != UNIT_NONE);
    if (live[s] && first_live < 0) first_live = s;
  }
  if (first_live < 0) return;
  coop_stage_consts(env, frame + cb);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint32_t i = i0 + (live[s] ? s : first_live), o = ML1_SLOTS * s;
    const Fp* ch = b.chain + (size_t)CHAIN_WORDS * i;
    if (lane < 3) lds_store_fp(frame, o + ML1_RP + lane, ch[CH_RP + lane]);
    else if (lane < 7) lds_store_fp(frame, o + ML1_HQ + lane - 3, ch[CH_HQ + lane - 3]);
  }
  if (lane == 0) *flag = 0;
  __syncthreads();
  coop_run(env, ml, frame, frame + cb, flag);
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (live[s] && lane < 12) reinterpret_cast<Fp*>(&b.f[i0 + s])[lane] = coop_get(frame, ML1_SLOTS * s + ML1_F + lane);
}

template <int S, class Lds>
__global__ __launch_bounds__(COOP_LANES) void k_mln(PipeBufs b, const CoopEnv* __restrict__ envp, uint32_t first, uint32_t count,
                                                    uint32_t units_paired) {
  const CoopEnv& env = *envp;
  __shared__ Lds sh;
  mln_items<S>(b, env, sh.frame, &sh.flag, (int)(sizeof(sh.frame) / sizeof(Fp)), first + (uint32_t)S * blockIdx.x,
               first + count, units_paired);
}

// The listed items' own single-pair loops, one wavefront each (a failing pass's later
// Miller loops, launch_k_mln_coop).
template <class Lds>
__global__ __launch_bounds__(COOP_LANES) void k_mln_items(PipeBufs b, const CoopEnv* __restrict__ envp,
                                                          const uint32_t* __restrict__ items) {
  __shared__ Lds sh;
  const uint32_t i = items[blockIdx.x];
  mln_items<1>(b, *envp, sh.frame, &sh.flag, (int)(sizeof(sh.frame) / sizeof(Fp)), i, i + 1, 0u);
}

// Sets per wavefront for a batch: 1 for small batches (latency: one set per two
// wavefronts spreads a small call over more SIMDs); from BLS_PACK_MIN_SETS sets on, 2
// while the process has at most $BLS_PACK3_INFLIGHT (2,048) sets in flight, else 3
// (three sets' steps share one wavefront's lanes: on the round-5 interpreter 1024-set
// calls at 4 x 1 / 8 x 1 / 12 x 1 contexts run 0.58M / 0.70M / 0.79M sets/s packed 3
// against 0.49-0.53M / 0.63-0.66M / 0.68-0.70M packed 2 and ~0.26M unpacked, but at
// 2 x 1 0.32M against 0.35M; profiles/r05_ab_perset_pack.json; round 4 had 2 ahead of 3
// everywhere).  $BLS_PACK (1, 2 or 3) forces a packing; $BLS_PACK_MIN overrides the
// threshold.
#define BLS_PACK_MIN_SETS 512u
static uint32_t pack_for(uint32_t n_sets) {
  static const int forced = [] {
    const char* e = getenv("BLS_PACK");
    return e ? atoi(e) : 0;
  }();
  static const uint32_t min_sets = [] {
    const char* e = getenv("BLS_PACK_MIN");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : BLS_PACK_MIN_SETS;
  }();
  if (forced >= 1 && forced <= 3) return (uint32_t)forced;
  static const uint64_t pack3_inflight = [] {
    const char* e = getenv("BLS_PACK3_INFLIGHT");
    return e ? (uint64_t)strtoull(e, nullptr, 10) : 2048ull;
  }();
  if (n_sets < min_sets) return 1u;
  return bls_sets_in_flight() > pack3_inflight ? 3u : 2u;
}

// The aggregated path's Miller loops are the SIMT pair k_mlq / k_mlf
// (kernels/k_mlq.hip); a test that forces a cooperative packing (BLS_DEBUG_PACK(1 / 2))
// runs them as the cooperative single-pair loops above instead, 1 or 2 per wavefront.
bool k_mln_list_ok(const PipeBufs& b) { return b.pack == 0 && b.ml_lines; }

hipError_t launch_k_mln_list(const PipeBufs& b, const uint32_t* items, uint32_t count, hipStream_t s) {
  if (count == 0) return hipSuccess;
  if (!k_mln_list_ok(b) || !items) return hipErrorInvalidValue;
  return launch_k_mlqf(b, 0, count, true, b.ml_lines, s, items);
}

// own_only: sets run their own Miller loop even when they belong to a unit (requests
// verified alone after their chunk failed)
hipError_t launch_k_mln(const PipeBufs& b, const CoopEnv& env, uint32_t first, uint32_t count, hipStream_t s,
                        bool own_only) {
  if (count == 0) return hipSuccess;
  if (b.pack == 0 && b.ml_lines) return launch_k_mlqf(b, first, count, own_only, b.ml_lines, s);
  const uint32_t up = own_only ? 0u : 1u;
  if (b.pack == 2 && env.ml1_2.n > 0) {
    k_mln<2, CoopLds><<<(count + 1) / 2, COOP_LANES, 0, s>>>(b, env.dev, first, count, up);
  } else {
    k_mln<1, CoopLds><<<count, COOP_LANES, 0, s>>>(b, env.dev, first, count, up);
  }
  return hipGetLastError();
}

// A failing pass's later Miller loops (chunk signature sums, the failed chunks' own loops,
// the individually verified requests' sums: items that never share f) as cooperative
// single-pair loops, one wavefront per item: ~1 ms of latency where the SIMT pair
// k_mlq + k_mlf2 takes ~7 ms (2.6 + 4.6; profiles/r05_cfg5_fallback.json "step3"), and the
// items are few.  Up to $BLS_COOP_ML_MAX items (default 8192; 0 turns it off); 0 items
// or no ml1_1 program: hipErrorNotSupported (the caller takes the SIMT pair).
uint32_t coop_ml_max() {
  static const uint32_t v = [] {
    const char* e = getenv("BLS_COOP_ML_MAX");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : 8192u;
  }();
  return v;
}

hipError_t launch_k_mln_coop(const PipeBufs& b, const CoopEnv& env, uint32_t first, uint32_t count,
                             const uint32_t* items, hipStream_t s) {
  if (count == 0) return hipSuccess;
  if (env.ml1_1.n == 0 || count > coop_ml_max()) return hipErrorNotSupported;
  if (items) k_mln_items<CoopLds><<<count, COOP_LANES, 0, s>>>(b, env.dev, items);
  else k_mln<1, CoopLds><<<count, COOP_LANES, 0, s>>>(b, env.dev, first, count, 0u);
  return hipGetLastError();
}

hipError_t launch_k_pset(const PipeBufs& b, const CoopEnv& env, hipStream_t s) {
  const uint32_t S = (b.pack >= 1 && b.pack <= 3) ? b.pack : pack_for(b.n_sets);
  if (S == 3 && env.packed[1].ml2.n > 0) {
    k_psetn<3, COOP_FRAME3><<<(b.n_sets + 2) / 3, COOP_LANES, 0, s>>>(b, env.dev);
  } else if (S == 2 && env.packed[0].ml2.n > 0) {
    k_psetn<2, COOP_FRAME2><<<(b.n_sets + 1) / 2, COOP_LANES, 0, s>>>(b, env.dev);
  } else {
    k_pset<<<b.n_sets, PSET_WAVES * COOP_LANES, 0, s>>>(b, env.dev);
  }
  return hipGetLastError();
}
