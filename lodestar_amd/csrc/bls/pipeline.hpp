// Per-thread stage bodies of the batch-verify pipeline, shared by the HIP kernels
// (lodestar_amd/csrc/bls_gpu.hip: one lane per set / request / chunk) and the CPU
// test harness (tests/native/hostsim.cpp, which loops the same bodies).
//
// Semantics follow the reference worker (beacon-node/src/chain/bls/multithread/
// worker.ts:32-108) and verifySignatureSetsMaybeBatch (chain/bls/maybeBatch.ts:16-39):
//   stage_pk          deserializeSet / getAggregatedPubkey      (worker.ts:110-116, utils.ts:5-16)
//   stage_sig         Signature.fromBytes(sig, affine, true)    (maybeBatch.ts:23,36)
//   stage_h2c         hash_to_G2(signingRoot)                   ([ext] blst)
//   stage_scale       r_i * pk_i, r_i * sig_i, 64-bit r_i       ([ext] verifyMultipleSignatures)
//   stage_pair_set    f_i = ML(r_i pk_i, H(m_i)) * ML(-g1, r_i sig_i)
//   stage_req_status  per-request error precedence              (worker.ts:45, maybeBatch.ts:16-39)
//   stage_chunk       FE(prod f_i) == 1 per chunk of >= 16 requests
//   stage_indiv       the same per request (fallback / non-batchable, worker.ts:76-98)
// The check prod e(r_i pk_i, H_i) * e(-g1, sum r_i sig_i) == 1 of the reference is
// evaluated with the -g1 pairing split per set (bilinearity: identical verdict), so
// every set's pairing work is independent and no cross-set point sum is needed.
//
// The GPU verify path (bls_gpu.hip) runs the per-set part as
//   stage_pre (single lane: SSWU points, signature decoding)  ->  k_pset (one
//   wavefront per set, kernels/k_pset.hip)  ->  stage_exact_set for the rare sets
//   k_pset flags (exceptional point additions, infinity signatures);
// the host harness runs the straight stages above, which compute the same values.
#pragma once

#include "../../../include/lodestar_bls.h"
#include "hash_to_curve.hpp"
#include "pairing.hpp"

namespace bls {

// Aggregated-signature path (bls_gpu.hip): k_chain -> k_gsum / k_vset -> k_mln hand-off
// per set, CHAIN_WORDS Fp: HQ = affine H(m) (x.c0, x.c1, y.c0, y.c1), RP = [r] pk
// (G1 Jacobian), RS = [r] sig (G2 Jacobian x.c0, x.c1, y.c0, y.c1, z.c0, z.c1).
// A group's virtual set (index n_sets + chunk, n_sets + n_chunks + individual
// request) holds HQ = affine(sum of the group's RS) and RP = -g1.
enum : int { CH_HQ = 0, CH_RP = 4, CH_RS = 7, CHAIN_WORDS = 13 };
#define UNIT_NONE 0xFFFFFFFFu

struct PipeBufs {
  uint32_t n_sets, n_reqs, n_chunks, n_indiv;
  // inputs
  const uint32_t* req_off;     // n_reqs + 1
  const uint8_t* pubkeys;      // raw mode: n_sets * 96
  const uint32_t* set_pk_off;  // table mode (nullable)
  const uint32_t* pk_idx;
  const G1A* pk_table;
  uint32_t pk_table_n;
  // aggregate sets of >= agg_min keys (0: none) are summed one wavefront per set by
  // k_pk_agg (a lane per key stride, then a tree over the lanes); stage_pk skips them
  const uint32_t* agg_sets;    // n_agg set indices
  uint32_t n_agg, agg_min;
  const uint8_t* msgs;         // n_sets * 32
  const uint8_t* sigs;         // n_sets * 96
  const uint32_t* sig_lens;    // nullable
  const uint32_t* seed;        // 8 words
  // signing-root dedup (nullable; plan_msg_dedup): SSWU points are computed once
  // per distinct 32-byte root and shared by every set signing that root
  const uint32_t* msg_uniq;    // n_uniq set indices: the first set of each distinct root
  const uint32_t* msg_rep;     // n_sets: the set whose SSWU points set i shares
  uint32_t n_uniq;
  uint32_t scalar_base;        // set i draws r from index scalar_base + i (shards of one call, bls_gpu_partial)
  uint32_t pack;               // sets per wavefront of k_pset (0: by call size; BLS_DEBUG_PACK)
  uint32_t mlf_pl;             // items per k_mlf lane (0: by the sets in flight; BLS_DEBUG_MLF_PL)
  uint32_t multi_set_rules;    // a shard of a larger call (bls_gpu_partial): no 1-set rules
  uint8_t* pk_inf;             // n_sets (nullable): 1 = the set's (aggregate) pubkey is infinity
  const uint32_t* chunk_off;   // n_chunks + 1 into chunk_reqs
  const uint32_t* chunk_reqs;
  const uint32_t* indiv_reqs;  // n_indiv
  const uint32_t* fold_groups; // n_fold [beg, end) pairs: k_fold multiplies f[beg + step], f[beg + 2 step].. < end into f[beg]
  uint32_t n_fold;
  uint32_t fold;               // stride of the folded f's an individual request multiplies (0 or 1: none)
  // intermediates
  G2A* sig;
  int32_t* sig_status;
  G1J* pk;
  int32_t* pk_status;
  // raw-pubkey calls: lowest set index whose 96-byte key failed to decode
  // (0xFFFFFFFF: none).  deserializeSet runs over every request of the worker
  // message before any verification and throws on the first bad key
  // (worker.ts:43-46), so the whole call rejects with that key's code.
  uint32_t* first_bad_pk;
  uint32_t* first_bad_pk_next;  // the next call's slot, reset by k_pk
  uint32_t init_set_flag;       // k_pk's initial set_flag (1: BLS_DEBUG_FORCE_EXACT)
  int32_t* req_status_host;     // host-mapped mirror of req_status (k_status), nullable
  uint32_t* flag_count_host;    // host-mapped copy of *flag_count (k_status), nullable
  G2A* H;
  G1J* rpk;
  G2J* rsig;
  Fp12* f;
  int32_t* req_status;
  Fp* q;               // n_sets * 8: the two SSWU points on E2' (x.c0, x.c1, y.c0, y.c1) per set
  // aggregated-signature path (sigagg = 1): f_i = ML(r_i pk_i, H_i) only, and per group
  // (chunk / individually verified request) one virtual set f = ML(-g1, sum r_i sig_i)
  // at n_sets + chunk / n_sets + n_chunks + t, multiplied in by the chunk, individual,
  // merged and partial products (kernels/k_fin.hip).  Sets the exact path finishes
  // keep both pairings in their own f_i and are left out of the sums.
  uint32_t sigagg;
  Fp* chain;             // (n_sets + virtual) * CHAIN_WORDS (layout: CH_*)
  uint32_t* chain_live;  // n_sets + virtual: 1 = k_mln runs this set's Miller loop
  uint8_t* chain_st;     // 4 n_sets: per set, role 0 H = O, role 1 outside G2, role 3 [r] pk = O
  G2J* rtab2;            // 15 n_sets: [1..15] sig per set (k_chain role 2's 4-bit window table)
  G1J* rtab1;            // 15 n_sets: [1..15] pk per set (role 3); per-set path: 30 n_sets (rpts)
  // per-set path (k_pset): RP = [s] pk at 2 i, RG = [s] g1 at 2 i + 1, made by k_pre's extra
  // lanes (kernels/k_pre.hip); nullable
  G1J* rpts;
  const uint32_t* gsets; // set indices of the groups being summed, group-major (k_gsum level 0)
  // Miller-loop units (sum r_i pk_i per signing root): with committee-shared
  // roots, the batchable sets of one chunk that sign the same root share ONE Miller loop
  // ML(sum r_i pk_i, H(root)) at f[unit_base + u]; such a set's own f_i is 1.
  // set_unit[i] = its unit or UNIT_NONE (own Miller loop); nullable (no units).
  const uint32_t* set_unit;
  const uint32_t* unit_off;  // n_chunks + 1: chunk c's units [unit_off[c], unit_off[c + 1])
  uint32_t unit_base, n_units;
  uint32_t indiv_vbase;      // f index of individually verified request t's signature sum
  // Shared Miller loops (k_mln, first pass): ml_dom[item] = the item's product domain
  // (its chunk, or 0x80000000 | request for a non-batchable request's sets); four
  // consecutive live items of one domain run ONE loop over their four pairs and keep
  // the product in the first item's f (the other three f = 1).  Nullable.
  const uint32_t* ml_dom;
  uint32_t* ml_lines;  // line buffer of the split SIMT Miller loops (k_mlq -> k_mlf), nullable
  uint32_t* set_flag;  // n_sets: 1 = take the exact single-lane path (stage_exact_set)
  uint32_t* flag_count;  // 1 word: sets flagged by the cooperative kernel (GPU path)
  // outputs
  int32_t* chunk_ok;       // n_chunks: 1 ok, 0 failed (retry)
  int32_t* indiv_verdict;  // n_indiv: 1 / 0 / -code (2: product left for the group tests)
  Fp12* chunk_fe;          // n_chunks: k_chunk_coop's final exponentiation (canonical), for
                           // the group tests' complement inference; nullptr: not kept
};

// Group tests over failed chunks' requests (bls_gpu.hip verify_groups; kernels/k_fin.hip):
// requests t >= n_direct of the indiv list leave their product F_t in f (no final
// exponentiation); k_group_coop checks FE(prod of the F_t of each group) == 1.  Kernel
// arguments of their own (only the two final-exponentiation kernels use them).
struct GroupBufs {
  uint32_t n_direct;
  Fp12* f;                   // n_indiv
  const uint32_t* off;       // n + 1
  const uint32_t* members;   // indices t into the indiv list
  uint32_t n;
  int32_t* verdict;          // n: 1 / 0 (host-mapped)
  // group sums (aggregated path): test g carries its own signature-sum pairing
  // ML(-g1, sum of its requests' r sig) in sum_f[g], and a group-tested request's F_t
  // holds its sets' f only; nullptr: each F_t holds its own request sum's pairing
  const Fp12* sum_f;
  // complement inference (bls_gpu.hip verify_groups): test g's final exponentiation kept
  // in fe[g] (canonical), and k_group_cmp sets bit 1 of verdict[g] when it equals that of
  // test ref[g] (its chunk's test of all requests; REF_NONE: none); fe nullptr: neither
  Fp12* fe;
  const uint32_t* ref;
  // ref[g] = REF_CHUNK | c: compare with chunk c's checked value ref_fe[c] instead
  const Fp12* ref_fe;
};
#define REF_CHUNK 0x80000000u
#define REF_NONE 0xFFFFFFFFu  // no comparison (the chunk indices stay far below 2^31 - 1)

BLS_HD void scalar_words_from_be32(const uint8_t* b, uint32_t k[8]) {
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = b + 28 - 4 * i;
    k[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
}

// r_i = first 8 bytes of SHA-256(seed || LE32(i)), forced non-zero
// (the reference draws randomBytesNonZero(8) per set, [ext] @chainsafe/blst).
BLS_HD uint64_t set_scalar(const uint32_t seed[8], uint32_t i) {
  uint32_t W[16];
  for (int k = 0; k < 8; ++k) W[k] = seed[k];
  W[8] = ((i & 0xffu) << 24) | (((i >> 8) & 0xffu) << 16) | (((i >> 16) & 0xffu) << 8) | (i >> 24);
  W[9] = 0x80000000u;
  for (int k = 10; k < 15; ++k) W[k] = 0;
  W[15] = 36 * 8;
  uint32_t s[8];
  sha256_init(s);
  sha256_compress(s, W);
  uint64_t r = ((uint64_t)s[0] << 32) | s[1];
  return r ? r : 1ull;
}

// *p = min(*p, v) (atomic on the device; the host harness runs lanes one by one)
BLS_HD void note_min_u32(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicMin(p, v);
#else
  if (v < *p) *p = v;
#endif
}

BLS_HD void stage_pk(const PipeBufs& b, uint32_t i) {
  if (i >= b.n_sets) return;
  int32_t code = BLS_OK;
  G1J acc = jac_infinity<Fp>();
  if (b.set_pk_off) {
    uint32_t beg = b.set_pk_off[i], end = b.set_pk_off[i + 1];
    if (b.agg_min && end - beg >= b.agg_min) return;  // k_pk_agg sums it
    if (beg == end) code = BLS_EMPTY_AGGREGATE;
    for (uint32_t k = beg; k < end; ++k) {
      uint32_t idx = b.pk_idx[k];
      if (idx >= b.pk_table_n) {
        code = BLS_BAD_ENCODING;
        break;
      }
      acc = jac_add_aff(acc, b.pk_table[idx]);
    }
  } else {
    G1A a;
    code = g1_deserialize96(b.pubkeys + 96ull * i, a);
    if (code == BLS_OK) acc = jac_from_aff(a);
    else if (b.first_bad_pk) note_min_u32(b.first_bad_pk, i);
  }
  b.pk[i] = acc;
  b.pk_status[i] = code;
  if (b.pk_inf) b.pk_inf[i] = (code == BLS_OK && jac_is_inf(acc)) ? 1 : 0;
}

BLS_HD void stage_sig(const PipeBufs& b, uint32_t i) {
  if (i >= b.n_sets) return;
  G2A s;
  s.inf = true;
  s.x = fp2_zero();
  s.y = fp2_zero();
  int32_t code;
  if (b.sig_lens && b.sig_lens[i] != 96) {
    code = BLS_INVALID_SIZE;
  } else {
    code = g2_decompress96(b.sigs + 96ull * i, s);
    if (code == BLS_OK && !g2_in_subgroup(s)) code = BLS_POINT_NOT_IN_GROUP;
  }
  b.sig[i] = s;
  b.sig_status[i] = code;
}

BLS_HD void stage_h2c(const PipeBufs& b, uint32_t i) {
  if (i >= b.n_sets) return;
  uint32_t w[8];
  msg_words_from_bytes(b.msgs + 32ull * i, w);
  b.H[i] = hash_to_g2(w);
}

BLS_HD void stage_scale(const PipeBufs& b, uint32_t i) {
  if (i >= b.n_sets) return;
  uint64_t r = set_scalar(b.seed, b.scalar_base + i);
  if (b.pk_status[i] == BLS_OK && b.sig_status[i] == BLS_OK) {
    b.rpk[i] = jac_mul_u64(b.pk[i], r);
    b.rsig[i] = aff_mul_u64(b.sig[i], r);
  } else {
    b.rpk[i] = jac_infinity<Fp>();
    b.rsig[i] = jac_infinity<Fp2>();
  }
}

BLS_HD G1Eval neg_g1_eval() {
  G1Eval ng1;
  ng1.xz = c_g1_x();
  ng1.y = c_g1_negy();
  ng1.z3 = c_one();
  return ng1;
}

// f_i = ML(r pk, H) * ML(-g1, r sig) (1 when the set's request errors anyway)
BLS_HD Fp12 pair_set(const G1J& rpk, const G2A& H, const G2J& rsig, bool sig_inf) {
  Fp12 f = miller_loop(g1_eval_from_jac(rpk), H);
  if (!sig_inf) f = fp12_mul(f, miller_loop(neg_g1_eval(), jac_to_aff(rsig)));
  return f;
}

BLS_HD void stage_pair_set(const PipeBufs& b, uint32_t i) {
  if (i >= b.n_sets) return;
  if (b.pk_status[i] == BLS_OK && b.sig_status[i] == BLS_OK && !jac_is_inf(b.rpk[i])) {
    b.f[i] = pair_set(b.rpk[i], b.H[i], b.rsig[i], b.sig[i].inf);
  } else {
    b.f[i] = fp12_one();
  }
}

// GPU pre-stage, one lane per task t in [0, pre_lanes(b)); u = distinct roots
// (n_uniq with dedup, else n_sets):
//   t < 2u:  SSWU point q_{t%2} of the set msg_uniq[t/2] (map_to_curve_sswu_fast;
//            on its rare false return the set is flagged for the exact path)
//   t >= pre_decode_base (2u rounded up to a wavefront): decode signature t - base
//            (on-curve, no subgroup test: k_pset does it)
// A group's signature sum s becomes its virtual set v for the Miller loops: HQ =
// affine(s) (one inversion), RP = -g1, so that f_v = ML(-g1, s); a sum at infinity (every
// set errored, or the sum cancels) leaves nothing to pair: f_v = 1 (k_vset, k_msm_window)
BLS_HD void vset_write(const PipeBufs& b, const G2J& s, uint32_t v) {
  if (jac_is_inf(s)) {
    b.chain_live[v] = 0u;
    Fp* d = reinterpret_cast<Fp*>(&b.f[v]);
    d[0] = c_one();
    for (int k = 1; k < 12; ++k) d[k] = fp_zero();
    return;
  }
  const Fp ni = fp_inv_gcd(fp_add(fp_sqr(s.z.c0), fp_sqr(s.z.c1)));
  const Fp2 zi = Fp2{fp_mul(s.z.c0, ni), fp_neg(fp_mul(s.z.c1, ni))};
  const Fp2 zi2 = fp2_sqr(zi);
  const Fp2 x = fp2_mul(s.x, zi2);
  const Fp2 y = fp2_mul(s.y, fp2_mul(zi2, zi));
  Fp* o = b.chain + (size_t)CHAIN_WORDS * v;
  o[CH_HQ + 0] = x.c0;
  o[CH_HQ + 1] = x.c1;
  o[CH_HQ + 2] = y.c0;
  o[CH_HQ + 3] = y.c1;
  o[CH_RP + 0] = c_g1_x();
  o[CH_RP + 1] = c_g1_negy();
  o[CH_RP + 2] = c_one();
  b.chain_live[v] = 1u;
}

BLS_HD uint32_t pre_roots(const PipeBufs& b) { return b.msg_uniq ? b.n_uniq : b.n_sets; }
// the decode lanes start at a wavefront boundary: a wavefront holding both kinds runs the
// SSWU chain and the decode chain one after the other (a 129-set block call's k_pre took
// 2.43 ms against 1.30 for 128 sets, profiles/r05_ab_pre_align.json)
BLS_HD uint32_t pre_decode_base(const PipeBufs& b) { return (2 * pre_roots(b) + 63u) & ~63u; }
BLS_HD uint32_t pre_lanes(const PipeBufs& b) { return pre_decode_base(b) + b.n_sets; }

BLS_HD void stage_pre(const PipeBufs& b, uint32_t t) {
  const uint32_t n = b.n_sets, u = pre_roots(b);
  if (t < 2 * u) {
    const uint32_t i = b.msg_uniq ? b.msg_uniq[t >> 1] : t >> 1;
    uint32_t w[8];
    msg_words_from_bytes(b.msgs + 32ull * i, w);
    Fp2 u0, u1;
    hash_to_field_fp2_x2(w, u0, u1);
    Fp2 x, y;
    Fp* q = b.q + 8ull * i + 4 * (t & 1);
    if (map_to_curve_sswu_fast((t & 1) ? u1 : u0, x, y)) {
      q[0] = x.c0;
      q[1] = x.c1;
      q[2] = y.c0;
      q[3] = y.c1;
    } else {
      b.set_flag[i] = 1u;
    }
    return;
  }
  const uint32_t base = pre_decode_base(b);
  if (t < base || t >= base + n) return;  // (the padding lanes before the decode lanes idle)
  const uint32_t i = t - base;
  G2A s;
  s.inf = true;
  s.x = fp2_zero();
  s.y = fp2_zero();
  int32_t code = (b.sig_lens && b.sig_lens[i] != 96) ? BLS_INVALID_SIZE : g2_decompress96(b.sigs + 96ull * i, s);
  b.sig[i] = s;
  b.sig_status[i] = code;
}

// After stage_pre with dedup: a set whose root is not the first of its kind takes
// the representative's SSWU points (and its exact-path flag), one lane per
// (set, Fp word) so the copy is coalesced.
BLS_HD void stage_qdup(const PipeBufs& b, uint32_t t) {
  const uint32_t i = t >> 3, k = t & 7;
  if (!b.msg_rep || i >= b.n_sets) return;
  const uint32_t r = b.msg_rep[i];
  if (r == i) return;
  b.q[8ull * i + k] = b.q[8ull * r + k];
  if (k == 0 && b.set_flag[r]) b.set_flag[i] = 1u;
}

// Exact per-set path for sets k_pset flagged: subgroup test, H(m), r pk, r sig and
// f_i with the complete (exception-handling) formulas of curve.hpp.
BLS_HD void stage_exact_set(const PipeBufs& b, uint32_t i) {
  if (i >= b.n_sets || !b.set_flag[i]) return;
  if (b.pk_status[i] != BLS_OK || b.sig_status[i] != BLS_OK || jac_is_inf(b.pk[i])) {
    b.f[i] = fp12_one();
    return;
  }
  const G2A sig = b.sig[i];
  if (!sig.inf && !g2_in_subgroup(sig)) {
    b.sig_status[i] = BLS_POINT_NOT_IN_GROUP;
    b.f[i] = fp12_one();
    return;
  }
  uint32_t w[8];
  msg_words_from_bytes(b.msgs + 32ull * i, w);
  const G2A H = hash_to_g2(w);
  const uint64_t r = set_scalar(b.seed, b.scalar_base + i);
  const G1J rpk = jac_mul_u64(b.pk[i], r);
  const G2J rsig = sig.inf ? jac_infinity<Fp2>() : aff_mul_u64(sig, r);
  b.f[i] = pair_set(rpk, H, rsig, sig.inf);
}

// The first code other than BLS_OK in s[beg, end) (in index order), or BLS_OK.  Eight
// loads per round with no early exit between them, so a 128-set request costs 16 load
// latencies instead of up to 128 dependent ones (k_status on the small-call path).
BLS_HD int32_t first_bad_status(const int32_t* s, uint32_t beg, uint32_t end) {
  for (uint32_t i = beg; i < end; i += 8) {
    int32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = i + k < end ? s[i + k] : BLS_OK;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (v[k] != BLS_OK) return v[k];
  }
  return BLS_OK;
}

// any Jacobian pubkey at infinity in pk[beg, end), four z's per round
BLS_HD bool any_pk_inf(const G1J* pk, uint32_t beg, uint32_t end) {
  for (uint32_t i = beg; i < end; i += 4) {
    bool inf[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) inf[k] = i + k < end && jac_is_inf(pk[i + k]);
    if (inf[0] || inf[1] || inf[2] || inf[3]) return true;
  }
  return false;
}

// Error precedence per request (r): pk decode / aggregation errors (deserializeSet
// runs first, worker.ts:45), then signature decode errors in set order
// (maybeBatch.ts:19-24 maps fromBytes over the sets), then the infinity rules
// of Signature.verify / verifyMultipleSignatures (oracle core_verify / verify_multiple).
BLS_HD void stage_req_status(const PipeBufs& b, uint32_t r) {
  if (r >= b.n_reqs) return;
  uint32_t beg = b.req_off[r], end = b.req_off[r + 1];
  int32_t code = BLS_OK;
  // a raw key that does not decode rejects every request of the call (worker.ts:45
  // throws out of verifyManySignatureSets; index.ts:367-374 rejects the whole group)
  const uint32_t bad = b.first_bad_pk ? *b.first_bad_pk : 0xFFFFFFFFu;
  if (bad != 0xFFFFFFFFu) {
    b.req_status[r] = b.pk_status[bad];
    return;
  }
  if (beg == end) code = BLS_EMPTY_SET;
  if (code == BLS_OK) code = first_bad_status(b.pk_status, beg, end);
  if (code == BLS_OK) code = first_bad_status(b.sig_status, beg, end);
  if (code == BLS_OK) {
    if (end - beg == 1 && !b.multi_set_rules) {
      if (b.sig[beg].inf) code = BLS_ZERO_SIGNATURE;
      else if (jac_is_inf(b.pk[beg])) code = BLS_PK_IS_INFINITY;
    } else if (any_pk_inf(b.pk, beg, end)) {
      code = BLS_PK_IS_INFINITY;
    }
  }
  b.req_status[r] = code;
}

BLS_HD void stage_chunk(const PipeBufs& b, uint32_t c) {
  if (c >= b.n_chunks) return;
  uint32_t beg = b.chunk_off[c], end = b.chunk_off[c + 1];
  for (uint32_t k = beg; k < end; ++k) {
    if (b.req_status[b.chunk_reqs[k]] != BLS_OK) {
      b.chunk_ok[c] = 0;  // the batch would throw -> retry every request (worker.ts:81-87)
      return;
    }
  }
  Fp12 F = fp12_one();
  for (uint32_t k = beg; k < end; ++k) {
    uint32_t r = b.chunk_reqs[k];
    for (uint32_t i = b.req_off[r]; i < b.req_off[r + 1]; ++i) F = fp12_mul(F, b.f[i]);
  }
  b.chunk_ok[c] = fp12_is_one(final_exponentiation(F)) ? 1 : 0;
}

BLS_HD void stage_indiv(const PipeBufs& b, uint32_t t) {
  if (t >= b.n_indiv) return;
  uint32_t r = b.indiv_reqs[t];
  int32_t code = b.req_status[r];
  if (code != BLS_OK) {
    b.indiv_verdict[t] = -code;
    return;
  }
  Fp12 F = fp12_one();
  const uint32_t stride = b.fold > 1 ? b.fold : 1u;
  for (uint32_t i = b.req_off[r]; i < b.req_off[r + 1]; i += stride) F = fp12_mul(F, b.f[i]);
  b.indiv_verdict[t] = fp12_is_one(final_exponentiation(F)) ? 1 : 0;
}

}  // namespace bls

// Host-side planning (plain host functions; parsed but not emitted in the device pass).
#include <stdlib.h>
#include <string.h>
#include <vector>

namespace bls {

// chunkifyMaximizeChunkSize (beacon-node/src/chain/bls/multithread/utils.ts:4-19)
static inline void chunkify_maximize_chunk_size(uint32_t n, uint32_t min_per_chunk, std::vector<uint32_t>& bounds) {
  bounds.clear();
  uint32_t chunk_count = n / min_per_chunk;
  bounds.push_back(0);
  if (chunk_count <= 1) {
    bounds.push_back(n);
    return;
  }
  uint32_t per = (n + chunk_count - 1) / chunk_count;
  for (uint32_t i = per; i < n; i += per) bounds.push_back(i);
  bounds.push_back(n);
}

// Host-side plan of one verify call: chunks over the batchable requests
// (BATCHABLE_MIN_PER_CHUNK = 16, worker.ts:17,56) and the non-batchable list.
struct BatchPlan {
  std::vector<uint32_t> chunk_off, chunk_reqs, nonbatch_reqs;
};

static inline void plan_batch(const bls_batch* in, BatchPlan& p) {
  std::vector<uint32_t> batchable;
  p.nonbatch_reqs.clear();
  for (uint32_t r = 0; r < in->n_reqs; ++r) {
    if (in->req_batchable && in->req_batchable[r]) batchable.push_back(r);
    else p.nonbatch_reqs.push_back(r);
  }
  p.chunk_off.clear();
  p.chunk_reqs = batchable;
  if (batchable.empty()) {
    p.chunk_off.push_back(0);
    return;
  }
  chunkify_maximize_chunk_size((uint32_t)batchable.size(), 16, p.chunk_off);
}

// Signing-root dedup for stage_pre: uniq = the first set of each distinct 32-byte
// root (in set order), rep[i] = that first set for set i.  Committee-shared roots
// (~512 attesters per root) then pay hash_to_field + SSWU once.
// Open addressing over a mix of all 32 bytes, so crafted roots cost probes, not
// wrong answers.  Returns the number of distinct roots.
static inline uint32_t plan_msg_dedup(const uint8_t* msgs, uint32_t n, std::vector<uint32_t>& uniq,
                                      std::vector<uint32_t>& rep) {
  uniq.clear();
  rep.resize(n);
  uint32_t cap = 16;
  while (cap < 2 * n) cap <<= 1;
  std::vector<uint32_t> slot(cap, 0xffffffffu);
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* m = msgs + 32ull * i;
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (int w = 0; w < 4; ++w) {
      uint64_t v;
      memcpy(&v, m + 8 * w, 8);
      h = (h ^ v) * 0xff51afd7ed558ccdull;
      h ^= h >> 32;
    }
    uint32_t pos = (uint32_t)h & (cap - 1);
    for (;;) {
      const uint32_t j = slot[pos];
      if (j == 0xffffffffu) {
        slot[pos] = i;
        rep[i] = i;
        uniq.push_back(i);
        break;
      }
      if (memcmp(msgs + 32ull * j, m, 32) == 0) {
        rep[i] = j;
        break;
      }
      pos = (pos + 1) & (cap - 1);
    }
  }
  return (uint32_t)uniq.size();
}

// Fill verdicts / stats from chunk results and the individual pass.
static inline void assemble_verdicts(const bls_batch* in, const BatchPlan& p, const int32_t* chunk_ok,
                                     const std::vector<uint32_t>& indiv_reqs, const int32_t* indiv_verdict,
                                     int32_t* verdicts, bls_stats* stats) {
  uint32_t n_chunks = (uint32_t)p.chunk_off.size() - 1;
  uint32_t retries = 0, sigs_ok = 0;
  for (uint32_t c = 0; c < n_chunks; ++c) {
    if (chunk_ok[c] == 1) {
      for (uint32_t k = p.chunk_off[c]; k < p.chunk_off[c + 1]; ++k) {
        uint32_t r = p.chunk_reqs[k];
        verdicts[r] = 1;
        sigs_ok += in->req_set_offsets[r + 1] - in->req_set_offsets[r];
      }
    } else {
      ++retries;
    }
  }
  for (size_t t = 0; t < indiv_reqs.size(); ++t) verdicts[indiv_reqs[t]] = indiv_verdict[t];
  if (stats) {
    stats->batch_retries = retries;
    stats->batch_sigs_success = sigs_ok;
    stats->n_chunks = n_chunks;
    stats->n_individual = (uint32_t)indiv_reqs.size();
  }
}

}  // namespace bls
