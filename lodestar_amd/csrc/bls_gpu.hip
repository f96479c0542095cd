// MI355X (gfx950) BLS12-381 signature-set verifier: host orchestration and the
// C-ABI declared in include/lodestar_bls.h.  Kernels: lodestar_amd/csrc/kernels/*.hip.
//
// Pipeline of one bls_gpu_verify call (one lane per set / request / chunk; the
// per-lane bodies live in bls/pipeline.hpp and are shared with the CPU test
// harness):
//   H2D (one packed copy from pinned staging)
//   k_pk     pubkey deserialize / device-table aggregation  -> G1 Jacobian
//   k_sig    signature decompress + G2 subgroup check       -> G2 affine + code
//   k_h2c    hash_to_G2(signing root)                       -> G2 affine
//   k_scale  r_i * pk_i (G1), r_i * sig_i (G2)
//   k_miller f_i = ML(r_i pk_i, H(m_i))
//   k_status per-request error precedence
//   k_chunk  per chunk of >= 16 batchable requests: prod f_i * ML(-g1, sum r_i sig_i), FE == 1
//   D2H chunk verdicts -> host plans the per-request fallback
//   k_indiv  failed chunks' requests + non-batchable requests, one lane each
// All kernels of a call run on the context's stream; the host waits twice
// (chunk verdicts, final verdicts).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <sys/random.h>

#include <vector>

#include "launchers.hpp"

using namespace bls;

struct bls_gpu_ctx {
  int device;
  hipStream_t stream;
  hipEvent_t ev0, ev1;
  hipEvent_t ev[9];  // stage boundaries of the last verify call
  char err[512];
  // device pubkey table (affine, Montgomery)
  G1A* table;
  uint32_t table_n, table_cap;
  // grow-only device workspace and pinned staging
  uint8_t* dev_ws;
  size_t dev_ws_cap;
  uint8_t* host_stage;
  size_t host_stage_cap;
};

static int set_err(bls_gpu_ctx* ctx, const char* what, hipError_t e) {
  if (ctx) snprintf(ctx->err, sizeof(ctx->err), "%s: %s", what, hipGetErrorString(e));
  return -1;
}

#define HIPC(ctx, call)                                     \
  do {                                                      \
    hipError_t e_ = (call);                                 \
    if (e_ != hipSuccess) return set_err((ctx), #call, e_); \
  } while (0)

// ---------------------------------------------------------------------------
// workspace helpers
// ---------------------------------------------------------------------------
namespace {

struct Carver {
  uint8_t* base;
  size_t off;
  template <class T>
  T* take(size_t count) {
    off = (off + 255) & ~(size_t)255;
    T* p = (T*)(base ? base + off : nullptr);
    off += sizeof(T) * (count ? count : 1);
    return p;
  }
};

int ensure_dev(bls_gpu_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->dev_ws_cap) return 0;
  if (ctx->dev_ws) HIPC(ctx, hipFree(ctx->dev_ws));
  ctx->dev_ws = nullptr;
  size_t cap = bytes + bytes / 4;
  HIPC(ctx, hipMalloc(&ctx->dev_ws, cap));
  ctx->dev_ws_cap = cap;
  return 0;
}

int ensure_host(bls_gpu_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->host_stage_cap) return 0;
  if (ctx->host_stage) HIPC(ctx, hipHostFree(ctx->host_stage));
  ctx->host_stage = nullptr;
  size_t cap = bytes + bytes / 4;
  HIPC(ctx, hipHostMalloc(&ctx->host_stage, cap, hipHostMallocDefault));
  ctx->host_stage_cap = cap;
  return 0;
}

// Copy a host array into the staging area at the same offset its device twin has.
template <class T>
void stage_copy(bls_gpu_ctx* ctx, const T* dev_ptr, const void* src, size_t bytes) {
  if (!src || !bytes) return;
  size_t off = (const uint8_t*)dev_ptr - ctx->dev_ws;
  memcpy(ctx->host_stage + off, src, bytes);
}

}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

int bls_gpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int bls_gpu_init(int device, bls_gpu_ctx** out) {
  *out = nullptr;
  bls_gpu_ctx* ctx = new bls_gpu_ctx();
  memset(ctx, 0, sizeof(*ctx));
  ctx->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    fprintf(stderr, "bls_gpu_init: hipSetDevice(%d): %s\n", device, hipGetErrorString(e));
    delete ctx;
    return -1;
  }
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
    delete ctx;
    return -1;
  }
  for (int i = 0; i < 9; ++i) {
    if (hipEventCreate(&ctx->ev[i]) != hipSuccess) {
      delete ctx;
      return -1;
    }
  }
  *out = ctx;
  return 0;
}

void bls_gpu_close(bls_gpu_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->table) (void)hipFree(ctx->table);
  if (ctx->dev_ws) (void)hipFree(ctx->dev_ws);
  if (ctx->host_stage) (void)hipHostFree(ctx->host_stage);
  (void)hipEventDestroy(ctx->ev0);
  (void)hipEventDestroy(ctx->ev1);
  for (int i = 0; i < 9; ++i) (void)hipEventDestroy(ctx->ev[i]);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* bls_gpu_last_error(const bls_gpu_ctx* ctx) { return ctx ? ctx->err : "no context"; }

int64_t bls_gpu_load_pubkeys(bls_gpu_ctx* ctx, const uint8_t* pks, uint32_t n, uint32_t pk_len, int32_t* codes) {
  if (pk_len != 48 && pk_len != 96) {
    snprintf(ctx->err, sizeof(ctx->err), "pk_len must be 48 or 96");
    return -1;
  }
  HIPC(ctx, hipSetDevice(ctx->device));
  if (ctx->table_n + n > ctx->table_cap) {
    uint32_t cap = (ctx->table_n + n) + (ctx->table_n + n) / 2 + 1024;
    G1A* t = nullptr;
    HIPC(ctx, hipMalloc(&t, sizeof(G1A) * (size_t)cap));
    if (ctx->table) {
      HIPC(ctx, hipMemcpyAsync(t, ctx->table, sizeof(G1A) * (size_t)ctx->table_n, hipMemcpyDeviceToDevice,
                               ctx->stream));
      HIPC(ctx, hipStreamSynchronize(ctx->stream));
      HIPC(ctx, hipFree(ctx->table));
    }
    ctx->table = t;
    ctx->table_cap = cap;
  }
  if (n == 0) return ctx->table_n;
  size_t in_bytes = (size_t)pk_len * n;
  Carver cv{nullptr, 0};
  cv.take<uint8_t>(in_bytes);
  cv.take<int32_t>(n);
  if (ensure_dev(ctx, cv.off) || ensure_host(ctx, cv.off)) return -1;
  Carver c2{ctx->dev_ws, 0};
  uint8_t* d_in = c2.take<uint8_t>(in_bytes);
  int32_t* d_codes = c2.take<int32_t>(n);
  HIPC(ctx, hipMemcpyAsync(d_in, pks, in_bytes, hipMemcpyHostToDevice, ctx->stream));
  HIPC(ctx, launch_k_load_pubkeys(d_in, n, pk_len, ctx->table + ctx->table_n, d_codes, ctx->stream));
  if (codes) HIPC(ctx, hipMemcpyAsync(codes, d_codes, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  ctx->table_n += n;
  return ctx->table_n;
}

int bls_gpu_verify(bls_gpu_ctx* ctx, const bls_batch* in, int32_t* verdicts, bls_stats* stats) {
  HIPC(ctx, hipSetDevice(ctx->device));
  const uint32_t n = in->n_sets, R = in->n_reqs;
  if (stats) memset(stats, 0, sizeof(*stats));
  if (R == 0) return 0;
  if (in->req_set_offsets[R] != n) {
    snprintf(ctx->err, sizeof(ctx->err), "req_set_offsets[n_reqs] != n_sets");
    return -2;
  }
  if (in->set_pk_offsets == nullptr && in->pubkeys == nullptr && n > 0) {
    snprintf(ctx->err, sizeof(ctx->err), "no pubkeys given");
    return -2;
  }
  BatchPlan plan;
  plan_batch(in, plan);
  const uint32_t n_chunks = (uint32_t)plan.chunk_off.size() - 1;
  const uint32_t n_pk_idx = in->set_pk_offsets ? in->set_pk_offsets[n] : 0;

  uint32_t seed_words[8];
  {
    uint8_t seed[32];
    if (in->seed) {
      memcpy(seed, in->seed, 32);
    } else if (getrandom(seed, 32, 0) != 32) {
      snprintf(ctx->err, sizeof(ctx->err), "getrandom failed");
      return -3;
    }
    scalar_words_from_be32(seed, seed_words);
  }

  // ---- carve the workspace: inputs first (one H2D copy), then intermediates
  auto carve = [&](Carver& c, PipeBufs& b, size_t& input_end) {
    b.req_off = c.take<uint32_t>(R + 1);
    b.chunk_off = c.take<uint32_t>(n_chunks + 1);
    b.chunk_reqs = c.take<uint32_t>(plan.chunk_reqs.size());
    b.seed = c.take<uint32_t>(8);
    b.pubkeys = in->set_pk_offsets ? nullptr : c.take<uint8_t>(96ull * n);
    b.set_pk_off = in->set_pk_offsets ? c.take<uint32_t>(n + 1) : nullptr;
    b.pk_idx = in->set_pk_offsets ? c.take<uint32_t>(n_pk_idx) : nullptr;
    b.msgs = c.take<uint8_t>(32ull * n);
    b.sigs = c.take<uint8_t>(96ull * n);
    b.sig_lens = in->signature_lens ? c.take<uint32_t>(n) : nullptr;
    b.indiv_reqs = c.take<uint32_t>(R);
    input_end = c.off;
    b.sig = c.take<G2A>(n);
    b.sig_status = c.take<int32_t>(n);
    b.pk = c.take<G1J>(n);
    b.pk_status = c.take<int32_t>(n);
    b.H = c.take<G2A>(n);
    b.rpk = c.take<G1J>(n);
    b.rsig = c.take<G2J>(n);
    b.f = c.take<Fp12>(n);
    b.req_status = c.take<int32_t>(R);
    b.chunk_ok = c.take<int32_t>(n_chunks);
    b.indiv_verdict = c.take<int32_t>(R);
  };
  PipeBufs b;
  memset(&b, 0, sizeof(b));
  size_t input_end = 0;
  {
    Carver c{nullptr, 0};
    carve(c, b, input_end);
    if (ensure_dev(ctx, c.off) || ensure_host(ctx, input_end)) return -1;
  }
  Carver c{ctx->dev_ws, 0};
  carve(c, b, input_end);
  b.n_sets = n;
  b.n_reqs = R;
  b.n_chunks = n_chunks;
  b.pk_table = ctx->table;
  b.pk_table_n = ctx->table_n;

  stage_copy(ctx, b.req_off, in->req_set_offsets, sizeof(uint32_t) * (R + 1));
  stage_copy(ctx, b.chunk_off, plan.chunk_off.data(), sizeof(uint32_t) * (n_chunks + 1));
  stage_copy(ctx, b.chunk_reqs, plan.chunk_reqs.data(), sizeof(uint32_t) * plan.chunk_reqs.size());
  stage_copy(ctx, b.seed, seed_words, sizeof(seed_words));
  if (b.pubkeys) stage_copy(ctx, b.pubkeys, in->pubkeys, 96ull * n);
  if (b.set_pk_off) {
    stage_copy(ctx, b.set_pk_off, in->set_pk_offsets, sizeof(uint32_t) * (n + 1));
    stage_copy(ctx, b.pk_idx, in->pk_indices, sizeof(uint32_t) * n_pk_idx);
  }
  stage_copy(ctx, b.msgs, in->messages, 32ull * n);
  if (in->signature_lens) {
    // bytes past a short signature's length are never read (the set fails INVALID_SIZE)
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t len = in->signature_lens[i] < 96 ? in->signature_lens[i] : 96;
      uint8_t* dst = ctx->host_stage + ((const uint8_t*)b.sigs - ctx->dev_ws) + 96ull * i;
      memset(dst, 0, 96);
      memcpy(dst, in->signatures + 96ull * i, len);
    }
    stage_copy(ctx, b.sig_lens, in->signature_lens, sizeof(uint32_t) * n);
  } else {
    stage_copy(ctx, b.sigs, in->signatures, 96ull * n);
  }

  hipStream_t s = ctx->stream;
  HIPC(ctx, hipEventRecord(ctx->ev0, s));
  HIPC(ctx, hipMemcpyAsync(ctx->dev_ws, ctx->host_stage, input_end, hipMemcpyHostToDevice, s));
  HIPC(ctx, hipEventRecord(ctx->ev[0], s));
  if (n > 0) {
    HIPC(ctx, launch_k_pk(b, s));
    HIPC(ctx, hipEventRecord(ctx->ev[1], s));
    HIPC(ctx, launch_k_sig(b, s));
    HIPC(ctx, hipEventRecord(ctx->ev[2], s));
    HIPC(ctx, launch_k_h2c(b, s));
    HIPC(ctx, hipEventRecord(ctx->ev[3], s));
    HIPC(ctx, launch_k_scale(b, s));
    HIPC(ctx, hipEventRecord(ctx->ev[4], s));
    HIPC(ctx, launch_k_miller(b, s));
    HIPC(ctx, hipEventRecord(ctx->ev[5], s));
  } else {
    for (int i = 1; i <= 5; ++i) HIPC(ctx, hipEventRecord(ctx->ev[i], s));
  }
  HIPC(ctx, launch_k_status(b, s));
  if (n_chunks > 0) HIPC(ctx, launch_k_chunk(b, s));
  HIPC(ctx, hipEventRecord(ctx->ev[6], s));

  std::vector<int32_t> chunk_ok(n_chunks + 1, 0);
  if (n_chunks > 0)
    HIPC(ctx, hipMemcpyAsync(chunk_ok.data(), b.chunk_ok, sizeof(int32_t) * n_chunks, hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipStreamSynchronize(s));

  std::vector<uint32_t> indiv = plan.nonbatch_reqs;
  for (uint32_t ch = 0; ch < n_chunks; ++ch)
    if (chunk_ok[ch] != 1)
      for (uint32_t k = plan.chunk_off[ch]; k < plan.chunk_off[ch + 1]; ++k) indiv.push_back(plan.chunk_reqs[k]);
  std::vector<int32_t> indiv_verdict(indiv.size() + 1, 0);
  if (!indiv.empty()) {
    b.n_indiv = (uint32_t)indiv.size();
    HIPC(ctx, hipMemcpyAsync((void*)b.indiv_reqs, indiv.data(), sizeof(uint32_t) * indiv.size(),
                             hipMemcpyHostToDevice, s));
    HIPC(ctx, hipEventRecord(ctx->ev[7], s));
    HIPC(ctx, launch_k_indiv(b, s));
    HIPC(ctx, hipEventRecord(ctx->ev[8], s));
    HIPC(ctx, hipMemcpyAsync(indiv_verdict.data(), b.indiv_verdict, sizeof(int32_t) * indiv.size(),
                             hipMemcpyDeviceToHost, s));
  }
  HIPC(ctx, hipEventRecord(ctx->ev1, s));
  HIPC(ctx, hipStreamSynchronize(s));
  assemble_verdicts(in, plan, chunk_ok.data(), indiv, indiv_verdict.data(), verdicts, stats);
  if (stats) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
    stats->device_ms = ms;
    // stage_ms: h2d, pk, sig, h2c, scale, miller, status+chunk, indiv
    (void)hipEventElapsedTime(&ms, ctx->ev0, ctx->ev[0]);
    stats->stage_ms[0] = ms;
    for (int i = 1; i <= 6; ++i) {
      (void)hipEventElapsedTime(&ms, ctx->ev[i - 1], ctx->ev[i]);
      stats->stage_ms[i] = ms;
    }
    stats->stage_ms[7] = 0.0;
    if (!indiv.empty()) {
      (void)hipEventElapsedTime(&ms, ctx->ev[7], ctx->ev[8]);
      stats->stage_ms[7] = ms;
    }
  }
  return 0;
}

int bls_gpu_aggregate_pubkeys(bls_gpu_ctx* ctx, const uint32_t* set_pk_offsets, const uint32_t* pk_indices,
                              uint32_t n_sets, uint8_t* out96, int32_t* codes) {
  HIPC(ctx, hipSetDevice(ctx->device));
  if (n_sets == 0) return 0;
  uint32_t n_idx = set_pk_offsets[n_sets];
  PipeBufs b;
  memset(&b, 0, sizeof(b));
  auto carve = [&](Carver& c, uint8_t*& d_out) {
    b.set_pk_off = c.take<uint32_t>(n_sets + 1);
    b.pk_idx = c.take<uint32_t>(n_idx);
    b.pk = c.take<G1J>(n_sets);
    b.pk_status = c.take<int32_t>(n_sets);
    d_out = c.take<uint8_t>(96ull * n_sets);
  };
  uint8_t* d_out = nullptr;
  {
    Carver c{nullptr, 0};
    carve(c, d_out);
    if (ensure_dev(ctx, c.off)) return -1;
  }
  Carver c{ctx->dev_ws, 0};
  carve(c, d_out);
  b.n_sets = n_sets;
  b.pk_table = ctx->table;
  b.pk_table_n = ctx->table_n;
  hipStream_t s = ctx->stream;
  HIPC(ctx, hipMemcpyAsync((void*)b.set_pk_off, set_pk_offsets, sizeof(uint32_t) * (n_sets + 1),
                           hipMemcpyHostToDevice, s));
  HIPC(ctx, hipMemcpyAsync((void*)b.pk_idx, pk_indices, sizeof(uint32_t) * n_idx, hipMemcpyHostToDevice, s));
  HIPC(ctx, launch_k_aggregate(b, d_out, s));
  HIPC(ctx, hipMemcpyAsync(out96, d_out, 96ull * n_sets, hipMemcpyDeviceToHost, s));
  if (codes) HIPC(ctx, hipMemcpyAsync(codes, b.pk_status, sizeof(int32_t) * n_sets, hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipStreamSynchronize(s));
  return 0;
}

static int run_simple(bls_gpu_ctx* ctx, uint32_t n, size_t in_a, const void* a, size_t in_b, const void* bsrc,
                      size_t out_per, void* out, int which) {
  HIPC(ctx, hipSetDevice(ctx->device));
  if (n == 0) return 0;
  size_t need = ((in_a * n + 255) & ~(size_t)255) + ((in_b * n + 255) & ~(size_t)255) + out_per * n + 256;
  if (ensure_dev(ctx, need)) return -1;
  Carver c{ctx->dev_ws, 0};
  uint8_t* d_a = c.take<uint8_t>(in_a * n);
  uint8_t* d_b = c.take<uint8_t>(in_b ? in_b * n : 1);
  uint8_t* d_o = c.take<uint8_t>(out_per * n);
  hipStream_t s = ctx->stream;
  HIPC(ctx, hipMemcpyAsync(d_a, a, in_a * n, hipMemcpyHostToDevice, s));
  if (in_b) HIPC(ctx, hipMemcpyAsync(d_b, bsrc, in_b * n, hipMemcpyHostToDevice, s));
  switch (which) {
    case 0: HIPC(ctx, launch_k_hash_to_g2(d_a, n, d_o, s)); break;
    case 1: HIPC(ctx, launch_k_sk_to_pk(d_a, n, d_o, s)); break;
    default: HIPC(ctx, launch_k_sign(d_a, d_b, n, d_o, s)); break;
  }
  HIPC(ctx, hipMemcpyAsync(out, d_o, out_per * n, hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipStreamSynchronize(s));
  return 0;
}

int bls_gpu_hash_to_g2(bls_gpu_ctx* ctx, const uint8_t* msgs, uint32_t n, uint8_t* out192) {
  return run_simple(ctx, n, 32, msgs, 0, nullptr, 192, out192, 0);
}

int bls_gpu_sk_to_pk(bls_gpu_ctx* ctx, const uint8_t* sks, uint32_t n, uint8_t* out48) {
  return run_simple(ctx, n, 32, sks, 0, nullptr, 48, out48, 1);
}

int bls_gpu_sign(bls_gpu_ctx* ctx, const uint8_t* sks, const uint8_t* msgs, uint32_t n, uint8_t* out96) {
  return run_simple(ctx, n, 32, sks, 32, msgs, 96, out96, 2);
}

}  // extern "C"

extern "C" int bls_gpu_mad_peak(bls_gpu_ctx* ctx, double* mads_per_s, double* ms_out) {
  HIPC(ctx, hipSetDevice(ctx->device));
  int cus = 0;
  HIPC(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
  const uint32_t blocks = (uint32_t)cus * 8, iters = 1024;
  if (ensure_dev(ctx, sizeof(uint64_t) * blocks)) return -1;
  uint64_t* d = (uint64_t*)ctx->dev_ws;
  hipStream_t s = ctx->stream;
  HIPC(ctx, launch_k_mad_peak(d, blocks, iters, s));  // warm-up (clocks, code load)
  HIPC(ctx, hipEventRecord(ctx->ev0, s));
  HIPC(ctx, launch_k_mad_peak(d, blocks, iters, s));
  HIPC(ctx, hipEventRecord(ctx->ev1, s));
  HIPC(ctx, hipStreamSynchronize(s));
  float ms = 0.f;
  HIPC(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  double mads = (double)blocks * 256.0 * iters * 16.0 * 8.0;
  *mads_per_s = mads / (ms * 1e-3);
  if (ms_out) *ms_out = ms;
  return 0;
}

extern "C" int bls_gpu_fp_mul_test(bls_gpu_ctx* ctx, const uint8_t* a48, const uint8_t* b48, uint32_t n,
                                   uint8_t* out48) {
  HIPC(ctx, hipSetDevice(ctx->device));
  if (n == 0) return 0;
  size_t sz = 48ull * n, al = (sz + 255) & ~(size_t)255;
  if (ensure_dev(ctx, 3 * al)) return -1;
  uint8_t *da = ctx->dev_ws, *db = da + al, *dout = db + al;
  hipStream_t s = ctx->stream;
  HIPC(ctx, hipMemcpyAsync(da, a48, sz, hipMemcpyHostToDevice, s));
  HIPC(ctx, hipMemcpyAsync(db, b48, sz, hipMemcpyHostToDevice, s));
  HIPC(ctx, launch_k_fp_mul_test(da, db, n, dout, s));
  HIPC(ctx, hipMemcpyAsync(out48, dout, sz, hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipStreamSynchronize(s));
  return 0;
}

// Dependent Montgomery-product chain: `lanes` lanes (multiple of 64) x `iters` products.
// ns_per_fpm = wall time / iters (per-lane latency); fpm_per_s = lanes * iters / time.
extern "C" int bls_gpu_fpm_bench(bls_gpu_ctx* ctx, uint32_t lanes, uint32_t iters, double* ns_per_fpm,
                                 double* fpm_per_s) {
  HIPC(ctx, hipSetDevice(ctx->device));
  lanes = (lanes + 63) / 64 * 64;
  if (ensure_dev(ctx, sizeof(Fp) * 2 * lanes)) return -1;
  Fp* io = (Fp*)ctx->dev_ws;
  hipStream_t s = ctx->stream;
  HIPC(ctx, hipMemsetAsync(io, 0x11, sizeof(Fp) * 2 * lanes, s));
  HIPC(ctx, launch_k_fpm_chain(io, lanes, 8, s));
  HIPC(ctx, hipEventRecord(ctx->ev0, s));
  HIPC(ctx, launch_k_fpm_chain(io, lanes, iters, s));
  HIPC(ctx, hipEventRecord(ctx->ev1, s));
  HIPC(ctx, hipStreamSynchronize(s));
  float ms = 0.f;
  HIPC(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  *ns_per_fpm = ms * 1e6 / iters;
  *fpm_per_s = (double)lanes * iters / (ms * 1e-3);
  return 0;
}
