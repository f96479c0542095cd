/*
 * lodestar_bls.h -- C-ABI of the MI355X BLS12-381 signature-set verifier.
 *
 * Drop-in boundary for Lodestar's BLS verification hot path.  The reference
 * crosses JS -> native inside @chainsafe/blst (SWIG N-API, [ext]); the seam this
 * library replaces is the worker RPC
 *     WorkerApi.verifyManySignatureSets(BlsWorkReq[]) -> BlsWorkResult
 * (packages/beacon-node/src/chain/bls/multithread/index.ts:59-61, worker.ts:26-108,
 *  types.ts:8-38), which sits behind
 *     IBlsVerifier.verifySignatureSets(sets, opts) (chain/bls/interface.ts:20-46).
 * The N-API binding a maintainer would add is shown in INTEGRATION.md.
 *
 * Conventions: plain pointers and sizes; the caller owns every buffer for the
 * duration of the call (the library copies into pinned staging); no call throws
 * across the ABI -- functions return 0 on success and a negative value on a
 * runtime failure (message via bls_gpu_last_error).  Per-request verdicts use
 *     1 = valid, 0 = invalid, < 0 = -(BLST-style error code)
 * with the codes below (values 1..7 follow blst's BLST_ERROR enum).
 */
#ifndef LODESTAR_BLS_H
#define LODESTAR_BLS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  BLS_CODE_OK = 0,
  BLS_CODE_BAD_ENCODING = 1,         /* "BLST_BAD_ENCODING" */
  BLS_CODE_POINT_NOT_ON_CURVE = 2,   /* "BLST_POINT_NOT_ON_CURVE" */
  BLS_CODE_POINT_NOT_IN_GROUP = 3,   /* "BLST_POINT_NOT_IN_GROUP" */
  BLS_CODE_PK_IS_INFINITY = 6,       /* "BLST_PK_IS_INFINITY" */
  BLS_CODE_INVALID_SIZE = 8,         /* "BLST_INVALID_SIZE" (multithread.test.ts:100) */
  BLS_CODE_ZERO_SIGNATURE = 9,       /* infinity signature on the 1-set path */
  BLS_CODE_EMPTY_SET = 10,           /* "Empty signature set" (maybeBatch.ts:29-31) */
  BLS_CODE_EMPTY_AGGREGATE = 11      /* "EMPTY_AGGREGATE_ARRAY" (PublicKey.aggregate([])) */
};

/* One verifyManySignatureSets() call: n_reqs BlsWorkReq, n_sets SerializedSet in
 * request order (types.ts:8-17).  Request r owns sets [req_set_offsets[r],
 * req_set_offsets[r+1]).  Public keys come either raw (96-byte uncompressed
 * affine, what index.ts:160 sends the worker) or as index lists into the
 * context's device-resident pubkey table (bls_gpu_load_pubkeys); an index list
 * of length k > 1 is an aggregate set, summed on the GPU (chain/bls/utils.ts:5-16). */
typedef struct bls_batch {
  uint32_t n_sets;
  uint32_t n_reqs;
  const uint32_t* req_set_offsets; /* n_reqs + 1 */
  const uint8_t* req_batchable;    /* n_reqs, 0/1 (VerifySignatureOpts.batchable) */
  const uint8_t* pubkeys;          /* n_sets * 96; used when set_pk_offsets == NULL */
  const uint32_t* set_pk_offsets;  /* n_sets + 1 into pk_indices, or NULL */
  const uint32_t* pk_indices;      /* device pubkey-table indices */
  const uint8_t* messages;         /* n_sets * 32 (signing roots) */
  const uint8_t* signatures;       /* n_sets * 96 (compressed G2; bytes past signature_lens[i] ignored) */
  const uint32_t* signature_lens;  /* n_sets, or NULL = all 96 */
  const uint8_t* seed;             /* 32 bytes for the random scalars, or NULL = fresh OS randomness */
} bls_batch;

/* BlsWorkResult bookkeeping (types.ts:26-38) */
typedef struct bls_stats {
  uint32_t batch_retries;      /* batchable chunks that failed and were re-verified per request */
  uint32_t batch_sigs_success; /* sets accepted by a successful batch */
  uint32_t n_chunks;           /* batchable chunks (chunkifyMaximizeChunkSize(reqs, 16)) */
  uint32_t n_individual;       /* requests verified on their own */
  uint32_t n_flagged;          /* sets finished by the exact single-lane path */
  double device_ms;            /* device time of the call (HIP events) */
  double stage_ms[8];          /* per stage (HIP events on the context's stream): h2d, pk, pre (SSWU + sig decode),
                                  k_chain (or k_pset), signature sums, Miller loops (k_mlq + k_mlf),
                                  status + merged / chunk checks, individual */
  uint32_t n_unique_msgs;      /* distinct signing roots hashed to the curve (== n_sets without dedup) */
  uint32_t merged_check;       /* 0 not run, 1 passed (per-chunk checks skipped), 2 failed (chunks checked),
                                  3 skipped: the context's previous pass failed it, chunks checked straight away */
  uint32_t n_ml_units;         /* Miller-loop units (chunk x shared signing root pairings), 0 = one per set */
  uint32_t pass_shape;         /* how the aggregated path ran (0 on the per-set path): bit 0 the merged signature
                                  sum by Pippenger MSM; bits 8-15 items per lane of the f side of the Miller loops
                                  (1, 2, 4; 3 = one item per two lanes) */
} bls_stats;

typedef struct bls_gpu_ctx bls_gpu_ctx;

/* Number of visible HIP devices (0 when there is no GPU). */
int bls_gpu_device_count(void);

/* Create a verifier bound to one device (one process per GPU; the device index is
 * local to the process).  Replaces BlsMultiThreadWorkerPool's worker creation
 * (multithread/index.ts:199-233). */
int bls_gpu_init(int device, bls_gpu_ctx** out);

/* The same with a stream priority: BLS_PRIORITY_HIGH puts the context's kernels ahead
 * of normal-priority contexts' queued work on the device -- the latency lane of
 * verifyOnMainThread calls (multithread/index.ts:138-151: the reference runs them on the
 * main thread, outside the worker queue).  BLS_PRIORITY_NORMAL = bls_gpu_init.
 *
 * Both admit a context only while the scratch the HIP runtime reserves for the
 * process's contexts fits a budget (see bls_admission below); otherwise they return
 * BLS_ERR_ADMISSION without creating anything, and bls_gpu_init_error() says why.  Any
 * other failure returns -1 (-2 for bad arguments) with its message there too.  The
 * reference's pool likewise records a worker that fails to start and keeps the others
 * (multithread/index.ts:221-229). */
#define BLS_PRIORITY_NORMAL 0
#define BLS_PRIORITY_HIGH 1
#define BLS_ERR_ADMISSION (-4)
int bls_gpu_init_priority(int device, int priority, bls_gpu_ctx** out);

/* Message of the last failed bls_gpu_init / bls_gpu_init_priority on the calling thread
 * ("" after a successful one). */
const char* bls_gpu_init_error(void);

/* Scratch admission.  The HIP runtime backs each hardware queue with private-segment
 * memory for a full device of the deepest kernel dispatched on it and aborts the queues
 * (HSA_STATUS_ERROR_OUT_OF_RESOURCES, every call of the process failing) past ~8 GiB.
 * A process's streams of one priority map onto at most GPU_MAX_HW_QUEUES hardware
 * queues (HIP's default 4), per priority level, so
 *   queues_in_use    = min(contexts_normal, hw_queues) + min(contexts_high, hw_queues)
 *   scratch_reserved = queues_in_use x scratch_per_queue
 * where scratch_per_queue is the deepest verify-path kernel's reservation (scratch
 * bytes per lane x 64 x resident waves per SIMD x 1024 SIMDs, from the kernels' resource
 * usage at build time; bls_scratch_worst_kernel names it).  A context is admitted while
 * scratch_reserved <= scratch_budget (default 6 GiB; $BLS_SCRATCH_BUDGET_MIB or
 * bls_gpu_set_scratch_budget). */
typedef struct bls_admission {
  uint32_t contexts_normal, contexts_high; /* open contexts on the device */
  uint32_t hw_queues;                      /* the runtime's hardware queues per priority (below) */
  uint32_t queues_in_use;
  uint64_t scratch_per_queue, scratch_reserved, scratch_budget; /* bytes */
  uint32_t hw_queues_known;                /* 1: hw_queues is the runtime's count (the variable's value when the
                                              runtime initialised under this library's first context, or the
                                              caller's argument); 0: unknown -- HIP was initialised before that
                                              context, hw_queues is the variable's value now (4 when unset);
                                              2: no context yet, hw_queues is what the runtime will read */
} bls_admission;

/* The accounting alone (no device needed): 0 if n_normal + n_high contexts are
 * admissible with hw_queues hardware queues per priority (0 = $GPU_MAX_HW_QUEUES), else
 * BLS_ERR_ADMISSION; *out (nullable) receives the figures. */
int bls_scratch_plan(uint32_t n_normal, uint32_t n_high, uint32_t hw_queues, bls_admission* out);
/* The figures for the contexts open on `device` now. */
int bls_gpu_admission(int device, bls_admission* out);
const char* bls_scratch_worst_kernel(void);
/* Override the budget for this process (0 restores the default / environment). */
void bls_gpu_set_scratch_budget(uint64_t bytes);

/* Ask the HIP runtime for n hardware queues per priority (one per verifier context, so
 * contexts do not serialise on HIP's default 4: 12 contexts x 22 calls run 2.27M sets/s
 * on 4 queues, 3.65M on 24).  The runtime reads GPU_MAX_HW_QUEUES once, when it
 * initialises; this sets the variable to n when it is unset and the runtime is not up
 * yet.  The library never writes the environment on its own: call this before any HIP
 * use in the process, from one thread (setenv).  Returns 0 applied, 1 left alone (the
 * variable is already set: the host's choice stands), 2 too late (the runtime is up and
 * keeps its count), -2 for n == 0.  The Python and JS wrappers call it (or set the
 * variable) as they load the library unless $BLS_KEEP_HW_QUEUES=1. */
int bls_gpu_request_hw_queues(uint32_t n);

/* Release device memory and streams (IBlsVerifier.close, index.ts:176-197). */
void bls_gpu_close(bls_gpu_ctx* ctx);

const char* bls_gpu_last_error(const bls_gpu_ctx* ctx);

/* Load / append trusted validator pubkeys into the device table (Index2PubkeyCache,
 * state-transition/src/cache/pubkeyCache.ts:56-77).  pk_len is 48 (compressed) or 96
 * (uncompressed).  codes (nullable, n entries) receive a per-key decode code; keys
 * are not subgroup-checked (trusted, pubkeyCache.ts:72-75).  All or nothing: when any
 * key fails to decode, no key is appended (the table keeps its size, so indices stay
 * aligned across contexts).  Returns the new table size (>= 0) or < 0 on failure. */
int64_t bls_gpu_load_pubkeys(bls_gpu_ctx* ctx, const uint8_t* pks, uint32_t n, uint32_t pk_len, int32_t* codes);

/* KeyValidate for n public keys (blst PublicKey.fromBytes(bytes, validate=true) [ext],
 * the check deposits get before a key enters the registry, state-transition
 * block/processDeposit.ts:56-65 -> index2pubkey, pubkeyCache.ts:56-77): decode
 * (48 compressed / 96 uncompressed), then BLST_PK_IS_INFINITY for the point at
 * infinity and BLST_POINT_NOT_IN_GROUP outside G1 (Scott's endomorphism test).
 * codes: n entries, 0 = valid.  Does not touch the device table. */
int bls_gpu_validate_pubkeys(bls_gpu_ctx* ctx, const uint8_t* pks, uint32_t n, uint32_t pk_len, int32_t* codes);

/* verifyManySignatureSets (worker.ts:32-108) on the GPU: per-request verdicts with
 * the reference's batch / fallback semantics:
 *   - batchable requests are grouped by chunkifyMaximizeChunkSize(reqs, 16) and each
 *     chunk is checked by one random-scalar batch (maybeBatch.ts:18-25);
 *   - a failing or erroring chunk is re-verified request by request;
 *   - non-batchable requests are verified on their own (maybeBatch.ts:16-39).
 * verdicts: n_reqs int32 (see top of file).  stats nullable. */
int bls_gpu_verify(bls_gpu_ctx* ctx, const bls_batch* batch, int32_t* verdicts, bls_stats* stats);

/* Several verifyManySignatureSets messages submitted together (the pool handing one
 * GPU context every message that is ready): the same verdicts and worker semantics as
 * n_batches bls_gpu_verify calls -- each message's batchable requests are chunked on
 * their own -- computed in one pass over the concatenated sets when every message
 * carries table-index pubkeys (messages with raw pubkeys run one after another).
 * verdicts: the messages' n_reqs entries concatenated; stats (nullable, one struct):
 * totals over the messages. */
int bls_gpu_verify_many(bls_gpu_ctx* ctx, const bls_batch* batches, uint32_t n_batches, int32_t* verdicts,
                        bls_stats* stats);

/* Sharded call across GPUs (north_star "each GPU reduces its shard to
 * an Fp12 partial, the partials are combined over RCCL/xGMI, and one final
 * exponentiation follows").  The reference verifies one call as ONE random-scalar
 * batch (maybeBatch.ts:18-25, blst verifyMultipleSignatures [ext]); here each rank
 * holds a contiguous shard of the call's sets and computes
 *     P_rank = prod_{i in shard} e(r_i pk_i, H(m_i)) e(-g1, r_i sig_i)   (Miller loops only)
 * with r_i drawn from the call's shared seed at index set_index_base + i, so the
 * scalars of all shards are distinct draws of one batch.  batch->seed must be set
 * (the same 32 bytes on every rank).  out576 receives P_rank as 12 Fp (opaque device
 * form: 12 x 48-byte Montgomery limbs; only bls_gpu_final_check reads it).  The shard is
 * verified with the rules of a multi-set call (no single-set rules, even for a 1-set
 * shard).  status: 0 if every set decoded, else -(code) of the shard's first error in
 * the reference's order -- class 0 a pubkey that does not decode / aggregate
 * (deserializeSet, worker.ts:45), class 1 a signature that does not decode
 * (maybeBatch.ts:19-24), class 2 an infinity pubkey -- and err_info (nullable,
 * 2 words) receives {class, shard-local set index} (class 3: none) so the ranks can
 * pick the call's first error; the whole call then rejects (rule 2 of SURVEY §8a) and
 * out576 is undefined.  The shard must hold >= 1 set. */
int bls_gpu_partial(bls_gpu_ctx* ctx, const bls_batch* batch, uint32_t set_index_base, uint8_t* out576,
                    int32_t* status, uint32_t* err_info, bls_stats* stats);

/* The combine step after the all-gather: *verdict = 1 iff FE(prod_k partials[k]) == 1,
 * one final exponentiation for the whole call (n >= 1 partials of 576 bytes). */
int bls_gpu_final_check(bls_gpu_ctx* ctx, const uint8_t* partials576, uint32_t n, int32_t* verdict);

/* getAggregatedPubkey (chain/bls/utils.ts:5-16) for n_sets index lists over the device
 * table; out: n_sets * 96 bytes uncompressed (PointFormat.uncompressed, index.ts:126,160);
 * codes: n_sets (0 ok, BLS_CODE_EMPTY_AGGREGATE for an empty list). */
int bls_gpu_aggregate_pubkeys(bls_gpu_ctx* ctx, const uint32_t* set_pk_offsets, const uint32_t* pk_indices,
                              uint32_t n_sets, uint8_t* out96, int32_t* codes);

/* G2 signature aggregation for the op pools:
 * Signature.aggregate(sigs.map((s) => Signature.fromBytes(s, undefined, true))) for each
 * of n_lists lists (aggregatedAttestationPool.ts:320-327 aggregateInto,
 * syncContributionAndProofPool.ts:181-185, syncCommitteeMessagePool.ts:122-129).
 * List l holds the 96-byte compressed signatures [list_offsets[l], list_offsets[l+1]).
 * out96: n_lists compressed sums; codes: 0, BLS_CODE_EMPTY_AGGREGATE for an empty list,
 * or the code of the list's first signature that does not decode / is outside G2. */
int bls_gpu_aggregate_signatures(bls_gpu_ctx* ctx, const uint8_t* sigs96, const uint32_t* list_offsets,
                                 uint32_t n_lists, uint8_t* out96, int32_t* codes);

/* Signature.fromBytes(bytes, CoordType.affine, validate) ([ext] @chainsafe/blst, as
 * maybeBatch.ts:23,36 call it): n 96-byte compressed G2 points -> out192 (uncompressed
 * ZCash order x.c1 || x.c0 || y.c1 || y.c0; the infinity encoding for the point at
 * infinity) and codes (0, or BLS_CODE_BAD_ENCODING / POINT_NOT_ON_CURVE /
 * POINT_NOT_IN_GROUP; the subgroup test only when validate != 0). */
int bls_gpu_g2_decompress(bls_gpu_ctx* ctx, const uint8_t* in96, uint32_t n, int validate, uint8_t* out192,
                          int32_t* codes);

/* hash_to_G2 with the POP DST for n 32-byte messages; out: n * 192 bytes (uncompressed
 * ZCash order x.c1 || x.c0 || y.c1 || y.c0). */
int bls_gpu_hash_to_g2(bls_gpu_ctx* ctx, const uint8_t* msgs, uint32_t n, uint8_t* out192);

/* SSZ object kinds of bls_gpu_ssz_roots: the fixed-size containers whose signing roots
 * the signature-set producers compute (state-transition/src/signatureSets/), given
 * in their SSZ serialization (fields concatenated, integers little-endian).  The value
 * is the serialized size in bytes in the low 8 bits. */
enum {
  BLS_SSZ_ROOT = 0x000 | 32,                /* Root / Bytes32: sync committee messages (block root), or an
                                               object root computed elsewhere (e.g. AggregateAndProof) */
  BLS_SSZ_UINT64 = 0x100 | 8,               /* Epoch / Slot: randao reveal, aggregate selection proof */
  BLS_SSZ_CHECKPOINT = 0x200 | 40,          /* Checkpoint{epoch, root} */
  BLS_SSZ_ATTESTATION_DATA = 0x300 | 128,   /* AttestationData: attestations, indexed attestations, slashings */
  BLS_SSZ_TWO_UINT64 = 0x400 | 16,          /* VoluntaryExit{epoch, validator_index},
                                               SyncAggregatorSelectionData{slot, subcommittee_index} */
  BLS_SSZ_BEACON_BLOCK_HEADER = 0x500 | 112, /* BeaconBlockHeader (== the block's root given its body root):
                                               proposer signatures, proposer slashings */
  BLS_SSZ_DEPOSIT_MESSAGE = 0x600 | 88,     /* DepositMessage{pubkey 48, withdrawal_credentials, amount} */
  BLS_SSZ_FORK_DATA = 0x700 | 36,           /* ForkData{current_version 4, genesis_validators_root}:
                                               computeForkDataRoot (util/domain.ts:40-45) */
  BLS_SSZ_SIGNING_DATA = 0x800 | 64         /* SigningData{object_root, domain} */
};
#define BLS_SSZ_SIZE(kind) ((uint32_t)(kind) & 0xFFu)

/* computeSigningRoot(type, obj, domain) (state-transition/src/util/signingRoot.ts:7-13)
 * for n serialized objects of one kind: out32[i] = hash_tree_root(SigningData{
 * hash_tree_root(obj_i), domain_i}); with domains == NULL, out32[i] = hash_tree_root(obj_i)
 * instead.  objs: n * BLS_SSZ_SIZE(kind) bytes; domain_stride 0 = one 32-byte domain for
 * every object, 32 = one per object.  Returns -2 for an unknown kind or stride. */
int bls_gpu_ssz_roots(bls_gpu_ctx* ctx, uint32_t kind, const uint8_t* objs, uint32_t n, const uint8_t* domains,
                      uint32_t domain_stride, uint8_t* out32);

/* Fixture helpers (signing is out of the verify path; used to synthesise inputs).
 * sks: n * 32 bytes big-endian scalars. */
int bls_gpu_sk_to_pk(bls_gpu_ctx* ctx, const uint8_t* sks, uint32_t n, uint8_t* out48);
int bls_gpu_sign(bls_gpu_ctx* ctx, const uint8_t* sks, const uint8_t* msgs, uint32_t n, uint8_t* out96);

/* Roofline probe: measured rate of v_mad_u64_u32 (32x32+64 multiply-add, the unit of
 * every Fp Montgomery product) on this device, with every CU at 8 waves/SIMD. */
int bls_gpu_mad_peak(bls_gpu_ctx* ctx, double* mads_per_s, double* ms);

/* Field self-test: out = a * b mod p for n pairs of canonical 48-byte big-endian
 * elements (exercises to/from Montgomery and the device Montgomery product). */
int bls_gpu_fp_mul_test(bls_gpu_ctx* ctx, const uint8_t* a48, const uint8_t* b48, uint32_t n, uint8_t* out48);

/* Probe: `lanes` lanes each run `iters` dependent Montgomery products. */
int bls_gpu_fpm_bench(bls_gpu_ctx* ctx, uint32_t lanes, uint32_t iters, double* ns_per_fpm, double* fpm_per_s);

/* Probe: time the cooperative (one wavefront per task) program `name` on `blocks`
 * tasks, `reps` runs each; us_per_step = run time / step count. */
int bls_gpu_coop_probe(bls_gpu_ctx* ctx, const char* name, uint32_t blocks, uint32_t reps, double* us_per_step,
                       double* ms_total,
                       uint64_t* step_stamps /* nullable, 2 n_steps + 1 s_memtime stamps (step start, compute done) */);

/* Design probe: launch the probe kernel `name` (kernels/k_probe.hip: "ml_simt_w1",
 * "ml_simt_w2", "fpm_d28") over `lanes` lanes `reps` times; *ms = wall time of the reps. */
int bls_gpu_kernel_probe(bls_gpu_ctx* ctx, const char* name, uint32_t lanes, uint32_t reps, double* ms);

/* Test hook: BLS_DEBUG_FORCE_EXACT routes every set through the exact single-lane
 * path (stage_exact_set) instead of the cooperative programs, so parity tests cover both. */
#define BLS_DEBUG_FORCE_EXACT 1u
/* Test / bench hook: compute hash_to_field + SSWU per set even when sets share a
 * signing root (the default dedups them, plan_msg_dedup in bls/pipeline.hpp). */
#define BLS_DEBUG_NO_MSG_DEDUP 2u
/* Test / bench hook: skip the merged check (one final exponentiation over every
 * chunk's sets before the per-chunk ones) and go straight to the chunk verdicts. */
#define BLS_DEBUG_NO_MERGED_CHECK 4u
/* Test / bench hook: sets per wavefront of the per-set cooperative kernel (1, 2 or 3;
 * 0 = by call size), so one process can run the same call through every packing. */
#define BLS_DEBUG_PACK(n) ((uint32_t)(n) << 8)
#define BLS_DEBUG_PACK_MASK 0x300u
/* Test / bench hook: force the aggregated-signature path (per-set chains one lane per
 * set, e(-g1, sum r_i sig_i) once per chunk, single-pair cooperative Miller loops) or
 * the all-cooperative per-set path; default: by call size (>= 512 sets: aggregated). */
#define BLS_DEBUG_SIGAGG_ON 8u
#define BLS_DEBUG_SIGAGG_OFF 16u
/* Test / bench hook: no Miller-loop units (one Miller loop per set even when sets of a
 * chunk share a signing root). */
#define BLS_DEBUG_NO_UNITS 32u
/* Test / bench hook: the merged signature sum as a Pippenger multi-scalar
 * multiplication (kernels/k_msm.hip) whatever $BLS_MSM says. */
#define BLS_DEBUG_MSM 64u
/* Test / bench hook: items per lane of the Miller loops' f side (1, 2 or 4; 3 = one item
 * per two lanes; 0 = by the process's sets in flight). */
#define BLS_DEBUG_MLF_PL(n) ((uint32_t)(n) << 12)
#define BLS_DEBUG_MLF_PL_MASK 0x7000u
/* Test / bench hook: group-test failed chunks of >= 4 requests whatever
 * $BLS_GROUP_TEST_MIN says (its default is 4 too; 0 turns group testing off). */
#define BLS_DEBUG_GROUP_TEST 128u
/* Test hook: run the merged check on every pass, also after a pass that failed it (by
 * default such a context's next pass checks its chunks straight away, merged_check 3). */
#define BLS_DEBUG_MERGED_EVERY_PASS 0x8000u
int bls_gpu_set_debug_flags(bls_gpu_ctx* ctx, uint32_t flags);

#ifdef __cplusplus
}
#endif

#endif /* LODESTAR_BLS_H */
