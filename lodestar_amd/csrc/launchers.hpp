// Host-side launchers, one per kernel translation unit (lodestar_amd/csrc/kernels/*.hip).
// Each heavy kernel lives in its own TU so the build compiles them in parallel.
#pragma once

#include <hip/hip_runtime.h>

#include "bls/pipeline.hpp"

#define BLS_BLOCK 64

// Serial tails of a pass (signature sums, their affine form, the product tree and the
// final exponentiations, status) run few wavefronts whose chains set the pass latency;
// with other passes' wide kernels on the same SIMDs they raise their wave priority so the
// SIMD issues them first (s_setprio 3; +3.6 % at 4 x 16, profiles/r03_ab_tail_prio.json).
#define BLS_TAIL_PRIO() __builtin_amdgcn_s_setprio(3)

static inline unsigned bls_grid_for(uint32_t n) { return (n + BLS_BLOCK - 1) / BLS_BLOCK; }

hipError_t launch_k_pk(const bls::PipeBufs& b, hipStream_t s);
hipError_t launch_k_pk_agg(const bls::PipeBufs& b, hipStream_t s);
#define BLS_AGG_WAVE_MIN 16u  // aggregate sets of at least this many keys: k_pk_agg
hipError_t launch_k_aggregate(const bls::PipeBufs& b, uint8_t* out96, hipStream_t s);
hipError_t launch_k_load_pubkeys(const uint8_t* pks, uint32_t n, uint32_t pk_len, bls::G1A* out, int32_t* codes,
                                 hipStream_t s);
hipError_t launch_k_status(const bls::PipeBufs& b, hipStream_t s);
hipError_t launch_k_validate_pubkeys(const uint8_t* pks, uint32_t n, uint32_t pk_len, int32_t* codes, hipStream_t s);
hipError_t launch_k_pre(const bls::PipeBufs& b, hipStream_t s);
hipError_t launch_k_exact(const bls::PipeBufs& b, hipStream_t s);
// roles: bit k runs k_chain role k (0 H, 1 subgroup, 2 [r] sig, 3 [r] pk); k_chain_done
// follows unless only role 2 runs (the merged check's fallback needs the per-set RS)
hipError_t launch_k_chain(const bls::PipeBufs& b, hipStream_t s, uint32_t roles = 0xFu);
// Pippenger sum of [r_i] sig_i over the live sets (kernels/k_msm.hip)
struct MsmBufs {
  uint32_t* cnt;      // 1020 bucket counts + 2 tickets: per context, zero between passes
  uint32_t* ticket;   // cnt + 1020
  uint32_t* off;      // 1021 bucket offsets into sorted
  uint32_t* seg_off;  // 1021 segment offsets
  uint32_t* ent;      // 8 n_sets (bucket << 22 | slot) entries
  uint32_t* sorted;   // 8 n_sets point references in bucket order
  bls::G2J* seg_sum;  // msm_seg_cap(n_sets)
  bls::G2J* bucket;   // 1020
  bls::G2J* win;      // 4
};
#define MSM_BUCKETS 1020u
size_t msm_seg_cap(uint32_t n_sets);
#define MSM_STATE_WORDS (MSM_BUCKETS + 2u)
// k_msm_bin: 22-bit bucket slots, <= 2 entries per set and bucket
#define MSM_MAX_SETS (1u << 21)
// mlf_per_lane(): one item per TWO f lanes (kernels/k_mlq.hip k_mlf2)
#define MLF_PAIR 3u
// the merged signature sum into the chunk groups' virtual sets vbase .. vbase + groups
hipError_t launch_k_msm(const bls::PipeBufs& b, const MsmBufs& m, uint32_t groups, uint32_t vbase, hipStream_t s);
hipError_t launch_k_gsum(const bls::PipeBufs& b, const uint32_t* seg, uint32_t n_seg, const bls::G2J* in,
                         bls::G2J* out, hipStream_t s);
hipError_t launch_k_vset(const bls::PipeBufs& b, const bls::G2J* sums, uint32_t n_groups, uint32_t vbase,
                         hipStream_t s);
hipError_t launch_k_gsum1(const bls::PipeBufs& b, const uint32_t* seg, uint32_t n_seg, const bls::G1J* in,
                          bls::G1J* out, hipStream_t s);
hipError_t launch_k_uset(const bls::PipeBufs& b, const bls::G1J* sums, const uint32_t* unit_rep, hipStream_t s);
#define GSUM_FAN 4u  // points per k_gsum segment (a 16-set chunk: two levels of 3 additions)
hipError_t launch_k_hash_to_g2(const uint8_t* msgs, uint32_t n, uint8_t* out192, hipStream_t s);
hipError_t launch_k_sig_aggregate(const uint8_t* in96, uint32_t n, const uint32_t* off, uint32_t n_lists,
                                  bls::G2A* pts, int32_t* sig_codes, uint8_t* out96, int32_t* codes, hipStream_t s);
hipError_t launch_k_g2_decompress(const uint8_t* in96, uint32_t n, int validate, uint8_t* out192, int32_t* codes,
                                  hipStream_t s);
hipError_t launch_k_ssz_roots(uint32_t kind, const uint8_t* objs, uint32_t n, const uint8_t* domains,
                              uint32_t domain_stride, uint8_t* out32, hipStream_t s);
bool ssz_kind_known(uint32_t kind);
hipError_t launch_k_sk_to_pk(const uint8_t* sks, uint32_t n, uint8_t* out48, hipStream_t s);
hipError_t launch_k_sign(const uint8_t* sks, const uint8_t* msgs, uint32_t n, uint8_t* out96, hipStream_t s);
hipError_t launch_k_mad_peak(uint64_t* out, uint32_t blocks, uint32_t iters, hipStream_t s);
hipError_t launch_k_fp_mul_test(const uint8_t* a, const uint8_t* b, uint32_t n, uint8_t* out, hipStream_t s);
hipError_t launch_k_fpm_chain(bls::Fp* io, uint32_t lanes, uint32_t iters, hipStream_t s);
size_t kernel_probe_out_bytes(const char* name);
hipError_t launch_kernel_probe(const char* name, void* out, uint32_t lanes, hipStream_t s);
#include "bls/coop.hpp"
hipError_t launch_k_chunk_coop(const bls::PipeBufs& b, const bls::CoopEnv& env, hipStream_t s);
hipError_t launch_k_indiv_coop(const bls::PipeBufs& b, const bls::CoopEnv& env, const bls::GroupBufs& g,
                              hipStream_t s);
hipError_t launch_k_group_coop(const bls::PipeBufs& b, const bls::CoopEnv& env, const bls::GroupBufs& g,
                              hipStream_t s);
hipError_t launch_k_fold(const bls::PipeBufs& b, const bls::CoopEnv& env, const uint32_t* groups, uint32_t n_groups,
                         uint32_t step, hipStream_t s);
// SIMT final exponentiations, one lane per chunk / request (kernels/k_fin_simt.hip), for
// a failing pass's many tasks: save = 4 Fp12 of device memory per task
uint32_t fe_simt_min();
hipError_t launch_k_chunk_simt(const bls::PipeBufs& b, bls::Fp12* save, hipStream_t s);
hipError_t launch_k_indiv_simt(const bls::PipeBufs& b, const bls::GroupBufs& g, bls::Fp12* save, hipStream_t s);
#define BLS_FOLD 16u  // sets per k_fold group (what k_indiv strides by)
#define BLS_FOLD1 4u  // sets per first-level k_fold group
hipError_t launch_k_coop_probe(const bls::CoopEnv& env, bls::CoopProg pg, uint32_t blocks, uint32_t reps,
                               uint32_t* sink, uint64_t* stamps, hipStream_t s);
#define FPROD_FAN 16u
hipError_t launch_k_fprod(const bls::Fp12* in, uint32_t n, bls::Fp12* out, int32_t* verdict,
                          const bls::CoopEnv& env, hipStream_t s);
hipError_t launch_k_pset(const bls::PipeBufs& b, const bls::CoopEnv& env, hipStream_t s);
hipError_t launch_k_mln(const bls::PipeBufs& b, const bls::CoopEnv& env, uint32_t first, uint32_t count,
                        hipStream_t s, bool own_only = false);
// own Miller loops of the listed items (items[0, count)) in one launch: the split SIMT
// kernels only (k_mln_list_ok); the individually verified pass uses it for every set of
// the failed chunks at once
bool k_mln_list_ok(const bls::PipeBufs& b);
hipError_t launch_k_mln_list(const bls::PipeBufs& b, const uint32_t* items, uint32_t count, hipStream_t s);
// cooperative single-pair loops of [first, first + count) or of items[0, count), one
// wavefront each, for a failing pass's later launches; hipErrorNotSupported above
// coop_ml_max() items (kernels/k_pset.hip)
hipError_t launch_k_mln_coop(const bls::PipeBufs& b, const bls::CoopEnv& env, uint32_t first, uint32_t count,
                             const uint32_t* items, hipStream_t s);
uint32_t coop_ml_max();
size_t mlq_line_words(uint32_t count);
// sets in the verify calls currently running in this process (every context)
uint64_t bls_sets_in_flight();
// items per lane of k_mlf (1, 2 or 4) for a launch now (kernels/k_mlq.hip)
uint32_t mlf_per_lane();
// ... and for a launch after the first pass (items that never share f), by its item count
uint32_t mlf_per_lane_alone(uint32_t count);
uint32_t mlf_per_lane_fixed();
uint64_t mlf_pair_max();
hipError_t launch_k_mlqf(const bls::PipeBufs& b, uint32_t first, uint32_t count, bool own_only, uint32_t* lines,
                         hipStream_t s, const uint32_t* items = nullptr);
