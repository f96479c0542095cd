/*
 * Thin N-API addon over the C-ABI of include/lodestar_bls.h: what Lodestar's
 * `GpuBlsVerifier` (integration/js/gpuBlsVerifier.js) loads in place of the
 * @chainsafe/blst worker pool (beacon-node/src/chain/bls/multithread/index.ts).
 *
 *   init(device, highPriority?) -> handle   (highPriority: bls_gpu_init_priority HIGH; throws an
 *          Error with code "BLS_ERR_ADMISSION" when the scratch admission refuses the context)
 *   loadPubkeys(handle, Uint8Array pks, pkLen) -> Int32Array codes
 *   verify(handle, {reqSetOffsets, reqBatchable, messages, signatures,
 *                   setPkOffsets?, pkIndices?, pubkeys?, signatureLens?, seed?})
 *          -> Promise<Int32Array verdicts>   (1 valid, 0 invalid, -code error)
 *   verifySync(handle, request) -> Int32Array   (the same on the calling thread)
 *   partial(handle, request, setIndexBase) -> Promise<{partial: Uint8Array(576) | null, status,
 *          errClass, errIndex}>   (bls_gpu_partial: a shard of a call split across devices;
 *          request.seed must hold the call's 32-byte seed)
 *   finalCheck(handle, Uint8Array partials (576 B each)) -> Promise<boolean>   (bls_gpu_final_check)
 *   close(handle)
 *
 * The verdict array carries the worker's BlsWorkResult bookkeeping (types.ts:26-38) as
 * properties: batchRetries, batchSigsSuccess, deviceMs, and workerStartNs / workerEndNs
 * (CLOCK_MONOTONIC ns as Numbers, the clock of process.hrtime.bigint(), taken on the
 * thread that ran the call) -- what the pool turns into its metrics
 * (multithread/index.ts:330-366: latencyToWorker, latencyFromWorker, batchRetries,
 * batchSigsSuccess, jobsWorkerTime).
 *
 * verify runs bls_gpu_verify on a libuv worker thread (napi_async_work): the JS
 * main thread never blocks on the GPU.  Input buffers are referenced until the
 * call completes (the library copies them into pinned staging at the start).
 *
 * Build (no node-gyp needed):
 *   gcc -O2 -shared -fPIC -I/usr/include/node -I include integration/napi/lodestar_bls_napi.c \
 *       -L lodestar_amd/_native -llodestar_bls -Wl,-rpath,'$ORIGIN' -o lodestar_amd/_native/lodestar_bls.node
 */
#define NAPI_VERSION 4
#include <execinfo.h>
#include <node_api.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "lodestar_bls.h"

#define CHECK(env, call)                                            \
  do {                                                              \
    if ((call) != napi_ok) {                                        \
      napi_throw_error((env), NULL, "lodestar_bls: N-API failure"); \
      return NULL;                                                  \
    }                                                               \
  } while (0)

/* One handle per JS verifier context.  Every entry point runs on the JS main thread
 * (verify_execute only touches ctx on a libuv worker), so the counters need no
 * locking.  close() while verifies are queued or running only marks the handle; the
 * last completing verify releases the device context.  Each queued job also holds a
 * reference to the handle object, so the GC finalizer cannot run under it; close()
 * removes the wrap, so a closed handle has no finalizer at all. */
typedef struct {
  bls_gpu_ctx* ctx;
  uint32_t inflight;
  int closed;
} bls_handle;

/* a closed handle with nothing in flight: release its device context and free it (the
 * caller does not touch h afterwards) */
static void handle_release_if_idle(bls_handle* h) {
  if (h->closed && h->inflight == 0) {
    if (h->ctx) bls_gpu_close(h->ctx);
    h->ctx = NULL;
    free(h);
  }
}

/* GC of a handle that was never closed (jobs hold a reference to the handle object, so
 * nothing is in flight then) */
static void handle_finalize(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  bls_handle* h = (bls_handle*)data;
  h->closed = 1;
  handle_release_if_idle(h);
}

static napi_value js_init(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int32_t dev = 0;
  bool high = false;
  if (argc > 0) CHECK(env, napi_get_value_int32(env, argv[0], &dev));
  if (argc > 1) {
    napi_valuetype t;
    CHECK(env, napi_typeof(env, argv[1], &t));
    if (t == napi_boolean) CHECK(env, napi_get_value_bool(env, argv[1], &high));
  }
  bls_gpu_ctx* ctx = NULL;
  const int rc = bls_gpu_init_priority(dev, high ? BLS_PRIORITY_HIGH : BLS_PRIORITY_NORMAL, &ctx);
  if (rc != 0 || !ctx) {
    /* the library's reason; error.code "BLS_ERR_ADMISSION" when the scratch admission
     * refused the context (the adapter then runs on the contexts it has, as the reference
     * pool keeps the workers that started, multithread/index.ts:221-229) */
    const char* why = bls_gpu_init_error();
    char msg[600];
    snprintf(msg, sizeof(msg), "%s", why && *why ? why : "bls_gpu_init failed (no HIP device?)");
    napi_throw_error(env, rc == BLS_ERR_ADMISSION ? "BLS_ERR_ADMISSION" : "BLS_ERR_INIT", msg);
    return NULL;
  }
  bls_handle* h = (bls_handle*)calloc(1, sizeof(bls_handle));
  h->ctx = ctx;
  /* the handle is a plain object wrapping h: close() removes the wrap, so a closed
   * handle leaves no finalizer for V8 to run at environment teardown (Node 12 ran such
   * finalizers during FreeEnvironment and crashed the process at exit, 1 run in ~3 of
   * the 16-context N-API bench; profiles/r06_napi_exit_crash.txt) */
  napi_value obj;
  CHECK(env, napi_create_object(env, &obj));
  if (napi_wrap(env, obj, h, handle_finalize, NULL, NULL) != napi_ok) {
    bls_gpu_close(ctx);
    free(h);
    napi_throw_error(env, NULL, "lodestar_bls: N-API failure");
    return NULL;
  }
  return obj;
}

/* the live handle behind v, or NULL (not a handle, or closed: use after close) */
static bls_handle* get_handle(napi_env env, napi_value v) {
  void* p = NULL;
  napi_valuetype t;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_object) return NULL;
  if (napi_unwrap(env, v, &p) != napi_ok || !p) return NULL;
  bls_handle* h = (bls_handle*)p;
  return h->closed ? NULL : h;
}

static napi_value js_close(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bls_handle* h = get_handle(env, argv[0]);
  if (h) {
    void* p = NULL;
    (void)napi_remove_wrap(env, argv[0], &p);  /* no finalizer from here on */
    h->closed = 1;
    handle_release_if_idle(h);  /* now, or when its last call completes */
  }
  return NULL;
}

/* typed array / buffer data pointer and byte length (NULL for undefined / null) */
static int view_of(napi_env env, napi_value v, void** data, size_t* bytes) {
  napi_valuetype t;
  *data = NULL;
  *bytes = 0;
  if (napi_typeof(env, v, &t) != napi_ok) return -1;
  if (t == napi_undefined || t == napi_null) return 0;
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (is_ta) {
    napi_typedarray_type tt;
    size_t len, off;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &tt, &len, data, &ab, &off) != napi_ok) return -1;
    size_t el = (tt == napi_uint32_array || tt == napi_int32_array) ? 4 : 1;
    *bytes = len * el;
    return 0;
  }
  return napi_get_buffer_info(env, v, data, bytes) == napi_ok ? 0 : -1;
}

static napi_value js_load_pubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bls_handle* h = get_handle(env, argv[0]);
  void* pks;
  size_t bytes;
  uint32_t pk_len = 48;
  if (!h || view_of(env, argv[1], &pks, &bytes)) {
    napi_throw_type_error(env, NULL, "loadPubkeys(handle, Uint8Array, pkLen)");
    return NULL;
  }
  if (argc > 2) CHECK(env, napi_get_value_uint32(env, argv[2], &pk_len));
  uint32_t n = (uint32_t)(bytes / pk_len);
  napi_value ab, out;
  void* codes;
  CHECK(env, napi_create_arraybuffer(env, 4 * (size_t)(n ? n : 1), &codes, &ab));
  CHECK(env, napi_create_typedarray(env, napi_int32_array, n, ab, 0, &out));
  if (bls_gpu_load_pubkeys(h->ctx, (const uint8_t*)pks, n, pk_len, (int32_t*)codes) < 0) {
    napi_throw_error(env, NULL, bls_gpu_last_error(h->ctx));
    return NULL;
  }
  return out;
}

enum { JOB_VERIFY = 0, JOB_PARTIAL = 1, JOB_FINAL = 2 };

typedef struct {
  int kind;
  bls_handle* h;
  bls_gpu_ctx* ctx;
  bls_batch batch;
  napi_ref keep;          /* the request object: keeps the input buffers alive */
  napi_ref keep_handle;   /* the handle object: no finalizer while the job is out */
  int32_t* verdicts;
  bls_stats stats;
  double t_start_ns, t_end_ns;
  int rc;
  /* JOB_PARTIAL / JOB_FINAL */
  uint32_t base;
  uint8_t part[576];
  int32_t status;
  uint32_t err_info[2];
  const uint8_t* partials;
  uint32_t n_partials;
  int32_t verdict;
  napi_deferred deferred;
  napi_async_work work;
} verify_job;

static double mono_ns(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e9 + (double)t.tv_nsec;
}

/* the BlsWorkResult bookkeeping as properties of the verdict array */
static void attach_stats(napi_env env, napi_value out, const bls_stats* st, double t0, double t1) {
  napi_value v;
  napi_create_uint32(env, st->batch_retries, &v);
  napi_set_named_property(env, out, "batchRetries", v);
  napi_create_uint32(env, st->batch_sigs_success, &v);
  napi_set_named_property(env, out, "batchSigsSuccess", v);
  napi_create_double(env, st->device_ms, &v);
  napi_set_named_property(env, out, "deviceMs", v);
  napi_create_double(env, t0, &v);
  napi_set_named_property(env, out, "workerStartNs", v);
  napi_create_double(env, t1, &v);
  napi_set_named_property(env, out, "workerEndNs", v);
}

static void verify_execute(napi_env env, void* data) {
  (void)env;
  verify_job* j = (verify_job*)data;
  j->t_start_ns = mono_ns();
  if (j->kind == JOB_PARTIAL)
    j->rc = bls_gpu_partial(j->ctx, &j->batch, j->base, j->part, &j->status, j->err_info, &j->stats);
  else if (j->kind == JOB_FINAL)
    j->rc = bls_gpu_final_check(j->ctx, j->partials, j->n_partials, &j->verdict);
  else
    j->rc = bls_gpu_verify(j->ctx, &j->batch, j->verdicts, &j->stats);
  j->t_end_ns = mono_ns();
}

static void verify_complete(napi_env env, napi_status status, void* data) {
  verify_job* j = (verify_job*)data;
  if (status != napi_ok || j->rc != 0) {
    napi_value msg, err;
    char text[640];
    snprintf(text, sizeof(text), "%s failed (rc %d, status %d): %s",
             j->kind == JOB_PARTIAL ? "bls_gpu_partial" : (j->kind == JOB_FINAL ? "bls_gpu_final_check" : "bls_gpu_verify"),
             j->rc, (int)status,
             j->rc ? bls_gpu_last_error(j->ctx) : "cancelled");
    napi_create_string_utf8(env, text, NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, j->deferred, err);
  } else if (j->kind == JOB_PARTIAL) {
    napi_value out, v;
    napi_create_object(env, &out);
    if (j->status == 0) {
      napi_value ab;
      void* dst;
      napi_create_arraybuffer(env, 576, &dst, &ab);
      memcpy(dst, j->part, 576);
      napi_create_typedarray(env, napi_uint8_array, 576, ab, 0, &v);
    } else {
      napi_get_null(env, &v);
    }
    napi_set_named_property(env, out, "partial", v);
    napi_create_int32(env, j->status, &v);
    napi_set_named_property(env, out, "status", v);
    napi_create_uint32(env, j->status ? j->err_info[0] : 3u, &v);
    napi_set_named_property(env, out, "errClass", v);
    napi_create_uint32(env, j->status ? j->err_info[1] : 0u, &v);
    napi_set_named_property(env, out, "errIndex", v);
    napi_create_double(env, j->t_start_ns, &v);
    napi_set_named_property(env, out, "workerStartNs", v);
    napi_create_double(env, j->t_end_ns, &v);
    napi_set_named_property(env, out, "workerEndNs", v);
    napi_resolve_deferred(env, j->deferred, out);
  } else if (j->kind == JOB_FINAL) {
    napi_value out;
    napi_get_boolean(env, j->verdict == 1, &out);
    napi_resolve_deferred(env, j->deferred, out);
  } else {
    napi_value ab, out;
    void* dst;
    uint32_t n = j->batch.n_reqs;
    napi_create_arraybuffer(env, 4 * (size_t)(n ? n : 1), &dst, &ab);
    memcpy(dst, j->verdicts, 4 * (size_t)n);
    napi_create_typedarray(env, napi_int32_array, n, ab, 0, &out);
    attach_stats(env, out, &j->stats, j->t_start_ns, j->t_end_ns);
    napi_resolve_deferred(env, j->deferred, out);
  }
  napi_delete_reference(env, j->keep);
  napi_delete_reference(env, j->keep_handle);
  napi_delete_async_work(env, j->work);
  j->h->inflight -= 1;
  handle_release_if_idle(j->h);
  free(j->verdicts);
  free(j);
}

static int prop(napi_env env, napi_value obj, const char* name, void** data, size_t* bytes) {
  napi_value v;
  if (napi_get_named_property(env, obj, name, &v) != napi_ok) return -1;
  return view_of(env, v, data, bytes);
}

/* Parse and check a request object into a bls_batch (buffers stay owned by the object). */
static int parse_request(napi_env env, napi_value req, bls_batch* b) {
  void *ro, *rb, *msg, *sig, *spo, *pki, *pks, *sl, *seed;
  size_t nro, nrb, nmsg, nsig, nspo, npki, npks, nsl, nseed;
  if (prop(env, req, "reqSetOffsets", &ro, &nro) || prop(env, req, "reqBatchable", &rb, &nrb) ||
      prop(env, req, "messages", &msg, &nmsg) || prop(env, req, "signatures", &sig, &nsig) ||
      prop(env, req, "setPkOffsets", &spo, &nspo) || prop(env, req, "pkIndices", &pki, &npki) ||
      prop(env, req, "pubkeys", &pks, &npks) || prop(env, req, "signatureLens", &sl, &nsl) ||
      prop(env, req, "seed", &seed, &nseed) || nro < 4 || !ro) {
    napi_throw_type_error(env, NULL, "verify: bad request object");
    return -1;
  }
  /* every buffer must hold what n_reqs / n_sets say: the library reads exactly that */
  const uint32_t n_reqs = (uint32_t)(nro / 4 - 1);
  const uint32_t n_sets = ((const uint32_t*)ro)[n_reqs];
  const size_t ns = n_sets;
  int ok = nrb >= n_reqs && nmsg >= 32 * ns && nsig >= 96 * ns && (!sl || nsl >= 4 * ns);
  if (spo) ok = ok && nspo >= 4 * (ns + 1) && npki >= 4 * (size_t)((const uint32_t*)spo)[n_sets];
  else ok = ok && pks && npks >= 96 * ns;
  if (!ok) {
    napi_throw_range_error(env, NULL, "verify: a buffer is shorter than n_reqs / n_sets require "
                                      "(pubkeys 96 B, messages 32 B, signatures 96 B per set)");
    return -1;
  }
  memset(b, 0, sizeof(*b));
  b->n_reqs = n_reqs;
  b->n_sets = n_sets;
  b->req_set_offsets = (const uint32_t*)ro;
  b->req_batchable = (const uint8_t*)rb;
  b->messages = (const uint8_t*)msg;
  b->signatures = (const uint8_t*)sig;
  b->set_pk_offsets = (const uint32_t*)spo;
  b->pk_indices = (const uint32_t*)pki;
  b->pubkeys = spo ? NULL : (const uint8_t*)pks;
  b->signature_lens = (const uint32_t*)sl;
  b->seed = nseed >= 32 ? (const uint8_t*)seed : NULL;
  return 0;
}

/* queue j on a libuv worker: keep = the object holding the input buffers */
static napi_value queue_job(napi_env env, bls_handle* h, verify_job* j, napi_value handle, napi_value keep) {
  j->h = h;
  j->ctx = h->ctx;
  napi_value promise, name;
  CHECK(env, napi_create_reference(env, keep, 1, &j->keep));
  CHECK(env, napi_create_reference(env, handle, 1, &j->keep_handle));
  CHECK(env, napi_create_promise(env, &j->deferred, &promise));
  CHECK(env, napi_create_string_utf8(env, "lodestar_bls_verify", NAPI_AUTO_LENGTH, &name));
  CHECK(env, napi_create_async_work(env, NULL, name, verify_execute, verify_complete, j, &j->work));
  CHECK(env, napi_queue_async_work(env, j->work));
  h->inflight += 1;
  return promise;
}

static napi_value js_verify(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bls_handle* h = argc >= 2 ? get_handle(env, argv[0]) : NULL;
  if (!h) {
    napi_throw_type_error(env, NULL, "verify(handle, request): no live handle (closed?)");
    return NULL;
  }
  bls_batch b;
  if (parse_request(env, argv[1], &b)) return NULL;
  verify_job* j = (verify_job*)calloc(1, sizeof(verify_job));
  j->kind = JOB_VERIFY;
  j->batch = b;
  j->verdicts = (int32_t*)calloc(b.n_reqs ? b.n_reqs : 1, 4);
  return queue_job(env, h, j, argv[0], argv[1]);
}

/* partial(handle, request, setIndexBase) -> Promise<{partial, status, errClass, errIndex}>:
 * bls_gpu_partial on a libuv worker -- one device's shard of a call split across the
 * devices of the node (gpuBlsVerifier.js splitCall). */
static napi_value js_partial(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bls_handle* h = argc >= 3 ? get_handle(env, argv[0]) : NULL;
  uint32_t base = 0;
  if (!h || napi_get_value_uint32(env, argv[2], &base) != napi_ok) {
    napi_throw_type_error(env, NULL, "partial(handle, request, setIndexBase): no live handle (closed?)");
    return NULL;
  }
  bls_batch b;
  if (parse_request(env, argv[1], &b)) return NULL;
  if (!b.seed || b.n_sets == 0) {
    napi_throw_range_error(env, NULL, "partial: the request needs >= 1 set and the call's 32-byte seed");
    return NULL;
  }
  verify_job* j = (verify_job*)calloc(1, sizeof(verify_job));
  j->kind = JOB_PARTIAL;
  j->batch = b;
  j->base = base;
  return queue_job(env, h, j, argv[0], argv[1]);
}

/* finalCheck(handle, partials) -> Promise<boolean>: FE(prod partials) == 1, bls_gpu_final_check. */
static napi_value js_final_check(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bls_handle* h = argc >= 2 ? get_handle(env, argv[0]) : NULL;
  void* p = NULL;
  size_t bytes = 0;
  if (!h || view_of(env, argv[1], &p, &bytes) || !p || bytes == 0 || bytes % 576) {
    napi_throw_type_error(env, NULL, "finalCheck(handle, Uint8Array of 576-byte partials)");
    return NULL;
  }
  verify_job* j = (verify_job*)calloc(1, sizeof(verify_job));
  j->kind = JOB_FINAL;
  j->partials = (const uint8_t*)p;
  j->n_partials = (uint32_t)(bytes / 576);
  return queue_job(env, h, j, argv[0], argv[1]);
}

/* verifySync(handle, request) -> Int32Array: the same call on the calling thread, for the
 * synchronous state-transition path (verifySignatureSet, state-transition
 * src/util/signatureSets.ts:24-38), which blocks the main thread as blst's verify does. */
static napi_value js_verify_sync(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bls_handle* h = argc >= 2 ? get_handle(env, argv[0]) : NULL;
  if (!h) {
    napi_throw_type_error(env, NULL, "verifySync(handle, request): no live handle (closed?)");
    return NULL;
  }
  bls_batch b;
  if (parse_request(env, argv[1], &b)) return NULL;
  napi_value ab, out;
  void* dst;
  CHECK(env, napi_create_arraybuffer(env, 4 * (size_t)(b.n_reqs ? b.n_reqs : 1), &dst, &ab));
  CHECK(env, napi_create_typedarray(env, napi_int32_array, b.n_reqs, ab, 0, &out));
  bls_stats st;
  const double t0 = mono_ns();
  if (bls_gpu_verify(h->ctx, &b, (int32_t*)dst, &st) != 0) {
    napi_throw_error(env, NULL, bls_gpu_last_error(h->ctx));
    return NULL;
  }
  attach_stats(env, out, &st, t0, mono_ns());
  return out;
}

/* sszRoots(handle, kind, objs, domains | null) -> Uint8Array(32 n): computeSigningRoot
 * (signingRoot.ts:7-13) for n serialized objects of one BLS_SSZ_* kind on the GPU;
 * domains: 32 bytes for all, 32 per object, or null for the hash_tree_roots.  Synchronous
 * (a few SHA-256 compressions per object). */
static napi_value js_ssz_roots(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bls_handle* h = argc >= 3 ? get_handle(env, argv[0]) : NULL;
  uint32_t kind = 0;
  void *objs = NULL, *doms = NULL;
  size_t ob = 0, db = 0;
  if (!h || napi_get_value_uint32(env, argv[1], &kind) != napi_ok || view_of(env, argv[2], &objs, &ob) ||
      (argc > 3 && view_of(env, argv[3], &doms, &db))) {
    napi_throw_type_error(env, NULL, "sszRoots(handle, kind, Uint8Array, domains)");
    return NULL;
  }
  const uint32_t size = BLS_SSZ_SIZE(kind);
  if (size == 0 || ob % size) {
    napi_throw_range_error(env, NULL, "sszRoots: objects are not a whole number of the kind's size");
    return NULL;
  }
  const uint32_t n = (uint32_t)(ob / size);
  uint32_t stride = 0;
  if (doms && db == 32ull * n && n != 1) stride = 32;
  else if (doms && db != 32) {
    napi_throw_range_error(env, NULL, "sszRoots: domains must be 32 bytes or 32 bytes per object");
    return NULL;
  }
  napi_value ab, out;
  void* roots;
  CHECK(env, napi_create_arraybuffer(env, 32 * (size_t)(n ? n : 1), &roots, &ab));
  CHECK(env, napi_create_typedarray(env, napi_uint8_array, 32 * (size_t)n, ab, 0, &out));
  if (bls_gpu_ssz_roots(h->ctx, kind, (const uint8_t*)objs, n, (const uint8_t*)doms, stride, (uint8_t*)roots) < 0) {
    napi_throw_error(env, NULL, bls_gpu_last_error(h->ctx));
    return NULL;
  }
  return out;
}

/* $BLS_NAPI_SEGV_TRACE=1 (diagnostics): a native backtrace on stderr if the process takes
 * SIGSEGV / SIGABRT / SIGBUS, then the default action; and a note when the process
 * reaches exit handlers, so a crash at exit can be placed */
static void segv_trace(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  static const char head[] = "lodestar_bls: fatal signal, native backtrace:\n";
  (void)!write(2, head, sizeof(head) - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
static void exit_note(void) {
  static const char msg[] = "lodestar_bls: exit handlers running\n";
  (void)!write(2, msg, sizeof(msg) - 1);
}

static napi_value module_init(napi_env env, napi_value exports) {
  const char* tr = getenv("BLS_NAPI_SEGV_TRACE");
  if (tr && *tr == '1') {
    signal(SIGSEGV, segv_trace);
    signal(SIGABRT, segv_trace);
    signal(SIGBUS, segv_trace);
    atexit(exit_note);
  }
  napi_property_descriptor d[] = {
      {"init", NULL, js_init, NULL, NULL, NULL, napi_default, NULL},
      {"close", NULL, js_close, NULL, NULL, NULL, napi_default, NULL},
      {"loadPubkeys", NULL, js_load_pubkeys, NULL, NULL, NULL, napi_default, NULL},
      {"verify", NULL, js_verify, NULL, NULL, NULL, napi_default, NULL},
      {"verifySync", NULL, js_verify_sync, NULL, NULL, NULL, napi_default, NULL},
      {"sszRoots", NULL, js_ssz_roots, NULL, NULL, NULL, napi_default, NULL},
      {"partial", NULL, js_partial, NULL, NULL, NULL, napi_default, NULL},
      {"finalCheck", NULL, js_final_check, NULL, NULL, NULL, napi_default, NULL},
  };
  napi_define_properties(env, exports, sizeof(d) / sizeof(d[0]), d);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, module_init)
