// Cooperative finalisation (one 64-lane wavefront per task; programs from
// tools/gen_coop.py, interpreter in bls/coop.hpp):
//   k_chunk_coop  one task per chunk of >= 16 batchable requests
//                 (worker.ts:56-88: random-scalar batch over the chunk's sets)
//   k_indiv_coop  one task per request verified on its own
//                 (failed chunks' requests and non-batchable requests, worker.ts:91-98);
//                 a failed chunk's requests under group testing only leave their product
//   k_group_coop  one task per group test: FE(prod of its requests' products) == 1
// Task: F = prod f_i, verdict = (FE(F) == 1).  Each f_i holds both pairings of its
// set (k_pset), or (aggregated-signature path, b.sigagg) only e(r pk, H) and the task
// multiplies in its group's virtual set ML(-g1, sum r_i sig_i).
#define BLS_FP_D28 1  // 28-bit-digit Montgomery product (bls/field.hpp)
#include "../launchers.hpp"
#include "../bls/coop.hpp"

using namespace bls;

typedef CoopLds FinShared;

__device__ void fin_accumulate_set(const PipeBufs& b, const CoopEnv& env, FinShared& sh, uint32_t i, bool& first) {
  if (first) {
    coop_load(sh.frame, FIN_F, reinterpret_cast<const Fp*>(&b.f[i]), 12);
    first = false;
    return;
  }
  coop_load(sh.frame, FIN_G, reinterpret_cast<const Fp*>(&b.f[i]), 12);
  coop_run(env, env.fin_fmul, sh.frame, sh.cbank, &sh.flag);
}

__device__ bool fin_finish(const CoopEnv& env, FinShared& sh) {
  coop_run(env, env.fin_fe1, sh.frame, sh.cbank, &sh.flag);
  coop_invert(sh.frame, FIN_INV_IN, FIN_INV_OUT);
  coop_run(env, env.fin_fe2, sh.frame, sh.cbank, &sh.flag);
  bool one = fp_eq(coop_get(sh.frame, FIN_F), c_one());
  for (int k = 1; k < 12; ++k) one = one && fp_is_zero(coop_get(sh.frame, FIN_F + k));
  return one;
}

__device__ void fin_init(const CoopEnv& env, FinShared& sh) {
  coop_stage_consts(env, sh.cbank);
  if (threadIdx.x < 12) lds_store_fp(sh.frame, FIN_F + threadIdx.x, threadIdx.x == 0 ? c_one() : fp_zero());
  if (threadIdx.x == 0) sh.flag = 0;
  __syncthreads();
}

__global__ __launch_bounds__(COOP_LANES) void k_chunk_coop(PipeBufs b, const CoopEnv* __restrict__ envp) {
  const CoopEnv& env = *envp;
  BLS_TAIL_PRIO();
  __shared__ FinShared sh;
  const uint32_t c = blockIdx.x;
  const uint32_t beg = b.chunk_off[c], end = b.chunk_off[c + 1];
  for (uint32_t k = beg; k < end; ++k) {
    if (b.req_status[b.chunk_reqs[k]] != BLS_OK) {
      if (threadIdx.x == 0) b.chunk_ok[c] = 0;  // the batch would throw -> retry (worker.ts:81-87)
      return;
    }
  }
  fin_init(env, sh);
  bool first = true;
  for (uint32_t k = beg; k < end; ++k) {
    const uint32_t r = b.chunk_reqs[k];
    for (uint32_t i = b.req_off[r]; i < b.req_off[r + 1]; ++i) {
      // a live set paired in its Miller-loop unit has f_i = 1: skip the product
      if (b.set_unit && b.set_unit[i] != UNIT_NONE && b.chain_live[i]) continue;
      fin_accumulate_set(b, env, sh, i, first);
    }
  }
  if (b.sigagg) fin_accumulate_set(b, env, sh, b.n_sets + c, first);  // ML(-g1, sum of the chunk's r sig)
  if (b.unit_off)
    for (uint32_t u = b.unit_off[c]; u < b.unit_off[c + 1]; ++u) fin_accumulate_set(b, env, sh, b.unit_base + u, first);
  bool ok = fin_finish(env, sh);
  if (b.chunk_fe && threadIdx.x < 12)
    reinterpret_cast<Fp*>(&b.chunk_fe[c])[threadIdx.x] = fp_reduce_once(coop_get(sh.frame, FIN_F + threadIdx.x));
  if (threadIdx.x == 0) b.chunk_ok[c] = ok ? 1 : 0;
}

__global__ __launch_bounds__(COOP_LANES) void k_indiv_coop(PipeBufs b, const CoopEnv* __restrict__ envp, GroupBufs gb) {
  const CoopEnv& env = *envp;
  BLS_TAIL_PRIO();
  __shared__ FinShared sh;
  const uint32_t t = blockIdx.x;
  const uint32_t r = b.indiv_reqs[t];
  const int32_t code = b.req_status[r];
  if (code != BLS_OK) {
    if (threadIdx.x == 0) b.indiv_verdict[t] = -code;
    return;
  }
  fin_init(env, sh);
  bool first = true;
  const uint32_t stride = b.fold > 1 ? b.fold : 1u;  // f's pre-multiplied in groups by k_fold
  for (uint32_t i = b.req_off[r]; i < b.req_off[r + 1]; i += stride) fin_accumulate_set(b, env, sh, i, first);
  // the request's own signature sum (a group-tested request under group sums: its tests'
  // sums instead, k_group_coop)
  if (b.sigagg && (t < gb.n_direct || !gb.sum_f)) fin_accumulate_set(b, env, sh, b.indiv_vbase + t, first);
  if (t >= gb.n_direct) {  // group-tested: the product only (k_group_coop)
    if (threadIdx.x < 12) reinterpret_cast<Fp*>(&gb.f[t])[threadIdx.x] = coop_get(sh.frame, FIN_F + threadIdx.x);
    if (threadIdx.x == 0) b.indiv_verdict[t] = 2;
    return;
  }
  bool ok = fin_finish(env, sh);
  if (threadIdx.x == 0) b.indiv_verdict[t] = ok ? 1 : 0;
}

// One group test: the requests' products (k_indiv_coop, indiv_f) multiplied, then one
// final exponentiation -- the same check as the requests' batch over their sets with the
// call's scalars (each product already holds both pairings of every set, or the
// request's own signature-sum pairing).
__global__ __launch_bounds__(COOP_LANES) void k_group_coop(const CoopEnv* __restrict__ envp, GroupBufs gb) {
  const CoopEnv& env = *envp;
  BLS_TAIL_PRIO();
  __shared__ FinShared sh;
  const uint32_t g = blockIdx.x;
  const uint32_t beg = gb.off[g], end = gb.off[g + 1];
  fin_init(env, sh);
  for (uint32_t k = beg; k < end; ++k) {
    const Fp* src = reinterpret_cast<const Fp*>(&gb.f[gb.members[k]]);
    if (k == beg) {
      coop_load(sh.frame, FIN_F, src, 12);
    } else {
      coop_load(sh.frame, FIN_G, src, 12);
      coop_run(env, env.fin_fmul, sh.frame, sh.cbank, &sh.flag);
    }
  }
  if (gb.sum_f) {  // the test's own signature-sum pairing (group sums)
    coop_load(sh.frame, FIN_G, reinterpret_cast<const Fp*>(&gb.sum_f[g]), 12);
    coop_run(env, env.fin_fmul, sh.frame, sh.cbank, &sh.flag);
  }
  bool ok = fin_finish(env, sh);
  if (gb.fe && threadIdx.x < 12)
    reinterpret_cast<Fp*>(&gb.fe[g])[threadIdx.x] = fp_reduce_once(coop_get(sh.frame, FIN_F + threadIdx.x));
  if (threadIdx.x == 0) gb.verdict[g] = ok ? 1 : 0;
}

// bit 1 of verdict[g]: FE of test g == FE of test ref[g], or of checked chunk
// ref[g] & ~REF_CHUNK (one lane per test, after k_group_coop in stream order)
__global__ __launch_bounds__(BLS_BLOCK) void k_group_cmp(GroupBufs gb) {
  const uint32_t g = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (g >= gb.n) return;
  const uint32_t r = gb.ref[g];
  if (r == REF_NONE) return;
  const Fp12* other = r < gb.n ? &gb.fe[r] : ((r & REF_CHUNK) && gb.ref_fe ? &gb.ref_fe[r & ~REF_CHUNK] : nullptr);
  if (!other) return;
  const uint32_t* a = reinterpret_cast<const uint32_t*>(&gb.fe[g]);
  const uint32_t* c = reinterpret_cast<const uint32_t*>(other);
  uint32_t diff = 0;
  for (int k = 0; k < 144; ++k) diff |= a[k] ^ c[k];
  if (diff == 0) gb.verdict[g] |= 2;
}

hipError_t launch_k_group_coop(const PipeBufs&, const CoopEnv& env, const GroupBufs& g, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  k_group_coop<<<g.n, COOP_LANES, 0, s>>>(env.dev, g);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !g.fe || !g.ref) return e;
  k_group_cmp<<<bls_grid_for(g.n), BLS_BLOCK, 0, s>>>(g);
  return hipGetLastError();
}

// Fold the f_i of individually verified requests in groups of b.fold consecutive sets
// (one wavefront per group, groups of all requests in parallel) so k_indiv_coop's
// sequential product over a large request (a 128-set block call: 127 Fp12 products)
// shrinks to one product per group.  Two launches: groups of BLS_FOLD1 consecutive f's
// (step 1), then groups of BLS_FOLD over those partial products (step BLS_FOLD1) -- 3 + 3
// products in a row per group of 16 instead of 15.
__global__ __launch_bounds__(COOP_LANES) void k_fold(PipeBufs b, const CoopEnv* __restrict__ envp,
                                                    const uint32_t* __restrict__ groups, uint32_t step) {
  const CoopEnv& env = *envp;
  BLS_TAIL_PRIO();
  __shared__ FinShared sh;
  const uint32_t beg = groups[2 * blockIdx.x], end = groups[2 * blockIdx.x + 1];
  if (end - beg <= step) return;
  fin_init(env, sh);
  coop_load(sh.frame, FIN_F, reinterpret_cast<const Fp*>(&b.f[beg]), 12);
  for (uint32_t k = beg + step; k < end; k += step) {
    coop_load(sh.frame, FIN_G, reinterpret_cast<const Fp*>(&b.f[k]), 12);
    coop_run(env, env.fin_fmul, sh.frame, sh.cbank, &sh.flag);
  }
  if (threadIdx.x < 12) reinterpret_cast<Fp*>(&b.f[beg])[threadIdx.x] = coop_get(sh.frame, FIN_F + threadIdx.x);
}

hipError_t launch_k_fold(const PipeBufs& b, const CoopEnv& env, const uint32_t* groups, uint32_t n_groups,
                         uint32_t step, hipStream_t s) {
  if (n_groups == 0) return hipSuccess;
  k_fold<<<n_groups, COOP_LANES, 0, s>>>(b, env.dev, groups, step);
  return hipGetLastError();
}

// Product tree over Fp12 values (sharded calls): block k multiplies
// in[k*FPROD_FAN .. min(n, (k+1)*FPROD_FAN)) into out[k].  With `verdict` non-null
// (one block, n <= FPROD_FAN) it runs the final exponentiation of the product
// instead and writes FE(prod) == 1.
__global__ __launch_bounds__(COOP_LANES) void k_fprod(const Fp12* in, uint32_t n, Fp12* out, int32_t* verdict,
                                                      const CoopEnv* __restrict__ envp) {
  const CoopEnv& env = *envp;
  BLS_TAIL_PRIO();
  __shared__ FinShared sh;
  const uint32_t beg = blockIdx.x * FPROD_FAN;
  const uint32_t end = beg + FPROD_FAN < n ? beg + FPROD_FAN : n;
  fin_init(env, sh);
  for (uint32_t k = beg; k < end; ++k) {
    // an exact 1 (the Miller-loop items whose product another item of their shared
    // loop holds: 7 of 8 sets of a chunk) leaves the product unchanged
    if (k != beg) {
      const Fp* src = reinterpret_cast<const Fp*>(&in[k]);
      const bool one = threadIdx.x >= 12 || fp_eq(src[threadIdx.x], threadIdx.x == 0 ? c_one() : fp_zero());
      if (__all(one)) continue;
    }
    coop_load(sh.frame, k == beg ? FIN_F : FIN_G, reinterpret_cast<const Fp*>(&in[k]), 12);
    if (k != beg) coop_run(env, env.fin_fmul, sh.frame, sh.cbank, &sh.flag);
  }
  if (verdict) {
    const bool ok = fin_finish(env, sh);
    if (threadIdx.x == 0) *verdict = ok ? 1 : 0;
  } else if (threadIdx.x < 12) {
    reinterpret_cast<Fp*>(&out[blockIdx.x])[threadIdx.x] = coop_get(sh.frame, FIN_F + threadIdx.x);
  }
}

hipError_t launch_k_fprod(const Fp12* in, uint32_t n, Fp12* out, int32_t* verdict, const CoopEnv& env,
                          hipStream_t s) {
  const uint32_t blocks = verdict ? 1u : (n + FPROD_FAN - 1) / FPROD_FAN;
  if (n == 0 || (verdict && n > FPROD_FAN)) return hipErrorInvalidValue;
  k_fprod<<<blocks, COOP_LANES, 0, s>>>(in, n, out, verdict, env.dev);
  return hipGetLastError();
}

hipError_t launch_k_chunk_coop(const PipeBufs& b, const CoopEnv& env, hipStream_t s) {
  k_chunk_coop<<<b.n_chunks, COOP_LANES, 0, s>>>(b, env.dev);
  return hipGetLastError();
}
// k_indiv_coop on two wavefronts per request: products, the easy part and the inversion
// on wavefront 0 (single-wavefront programs, block barriers between), the hard part
// (fin_fe2_w2) on both, so every product of its steps finds a lane pair -- for calls with
// few requests verified alone (a small non-batchable call's one request), where the
// final exponentiation is on the call's critical path.  Every branch reads block-uniform
// values.
__device__ void fin_accumulate_set2(const PipeBufs& b, const CoopEnv& env, FinShared& sh, uint32_t i, bool& first,
                                    bool w0) {
  if (first) {
    coop_load(sh.frame, FIN_F, reinterpret_cast<const Fp*>(&b.f[i]), 12);
    first = false;
    return;
  }
  coop_load(sh.frame, FIN_G, reinterpret_cast<const Fp*>(&b.f[i]), 12);
  if (w0) coop_run(env, env.fin_fmul, sh.frame, sh.cbank, &sh.flag);
  __syncthreads();
}

__global__ __launch_bounds__(2 * COOP_LANES) void k_indiv_coop2(PipeBufs b, const CoopEnv* __restrict__ envp,
                                                                GroupBufs gb) {
  const CoopEnv& env = *envp;
  BLS_TAIL_PRIO();
  __shared__ FinShared sh;
  const uint32_t t = blockIdx.x;
  const uint32_t r = b.indiv_reqs[t];
  const int32_t code = b.req_status[r];
  if (code != BLS_OK) {
    if (threadIdx.x == 0) b.indiv_verdict[t] = -code;
    return;
  }
  const bool w0 = threadIdx.x < COOP_LANES;
  fin_init(env, sh);
  bool first = true;
  const uint32_t stride = b.fold > 1 ? b.fold : 1u;
  for (uint32_t i = b.req_off[r]; i < b.req_off[r + 1]; i += stride) fin_accumulate_set2(b, env, sh, i, first, w0);
  if (b.sigagg && (t < gb.n_direct || !gb.sum_f)) fin_accumulate_set2(b, env, sh, b.indiv_vbase + t, first, w0);
  if (t >= gb.n_direct) {
    if (threadIdx.x < 12) reinterpret_cast<Fp*>(&gb.f[t])[threadIdx.x] = coop_get(sh.frame, FIN_F + threadIdx.x);
    if (threadIdx.x == 0) b.indiv_verdict[t] = 2;
    return;
  }
  if (w0) {
    coop_run(env, env.fin_fe1, sh.frame, sh.cbank, &sh.flag);
    coop_invert(sh.frame, FIN_INV_IN, FIN_INV_OUT);
  }
  __syncthreads();
  coop_run2_t(env, env.fin_fe2_w2, sh.frame, &sh.flag);
  bool one = fp_eq(coop_get(sh.frame, FIN_F), c_one());
  for (int k = 1; k < 12; ++k) one = one && fp_is_zero(coop_get(sh.frame, FIN_F + k));
  if (threadIdx.x == 0) b.indiv_verdict[t] = one ? 1 : 0;
}

// Up to $BLS_INDIV2_MAX (64) requests verified alone: two wavefronts each (k_indiv_coop2);
// more: one (the rate of a failing pass's many requests)
hipError_t launch_k_indiv_coop(const PipeBufs& b, const CoopEnv& env, const GroupBufs& g, hipStream_t s) {
  static const uint32_t w2_max = [] {
    const char* e = getenv("BLS_INDIV2_MAX");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : 64u;
  }();
  if (b.n_indiv <= w2_max && env.fin_fe2_w2.n > 0) k_indiv_coop2<<<b.n_indiv, 2 * COOP_LANES, 0, s>>>(b, env.dev, g);
  else k_indiv_coop<<<b.n_indiv, COOP_LANES, 0, s>>>(b, env.dev, g);
  return hipGetLastError();
}

// Probe: run program `pg` `reps` times on a block-private frame of pseudo-random
// field elements (timing of the interpreter; results discarded).
__global__ __launch_bounds__(COOP_LANES) void k_coop_probe(const CoopEnv* __restrict__ envp, CoopProg pg, uint32_t reps, uint32_t* sink,
                                                          uint64_t* stamps) {
  const CoopEnv& env = *envp;
  __shared__ CoopLdsN<COOP_FRAME3> sh;  // large enough for every program (1-, 2- and 3-set frames)
  coop_stage_consts(env, sh.cbank);
  for (int k = threadIdx.x; k < COOP_FRAME3; k += COOP_LANES) {
    Fp v = fp_zero();
    for (int i = 0; i < 11; ++i) v.l[i] = (uint32_t)(k * 2654435761u + i * 40503u + blockIdx.x);
    lds_store_fp(sh.frame, k, v);
  }
  if (threadIdx.x == 0) sh.flag = 0;
  __syncthreads();
  for (uint32_t r = 0; r < reps; ++r) coop_run(env, pg, sh.frame, sh.cbank, &sh.flag);
  if (threadIdx.x == 0 && sh.frame[0].l[0] == 0x12345678u) sink[blockIdx.x] = sh.flag;
  if (stamps && blockIdx.x == 0) coop_run_t<true>(env, pg, sh.frame, sh.cbank, &sh.flag, stamps);
}

hipError_t launch_k_coop_probe(const CoopEnv& env, CoopProg pg, uint32_t blocks, uint32_t reps, uint32_t* sink,
                               uint64_t* stamps, hipStream_t s) {
  k_coop_probe<<<blocks, COOP_LANES, 0, s>>>(env.dev, pg, reps, sink, stamps);
  return hipGetLastError();
}
