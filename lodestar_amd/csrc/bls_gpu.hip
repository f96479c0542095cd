// MI355X (gfx950) BLS12-381 signature-set verifier: host orchestration and the
// C-ABI declared in include/lodestar_bls.h.  Kernels: lodestar_amd/csrc/kernels/*.hip.
//
// Pipeline of one bls_gpu_verify call (single-lane bodies in bls/pipeline.hpp,
// shared with the CPU test harness; cooperative programs from tools/gen_coop.py):
//   H2D (one packed copy from pinned staging)
//   k_pk     pubkey deserialize / device-table aggregation   one lane per set
//   k_pre    SSWU points q0, q1 of H(m); signature decode    three lanes per set
//   k_pset   H(m), G2 subgroup test, r pk, r g1,             one wavefront per set
//            f_i = ML(r pk, H) ML(-r g1, sig)                 (k_psetn: 3 sets per wavefront
//                                                              from 512 sets per call)
//   (k_exact: complete formulas for the rare flagged sets, launched with a redo of
//    k_status / k_chunk only when k_pset counted any)
//   k_status per-request error precedence
//   k_chunk  per chunk of >= 16 batchable requests: FE(prod f_i) == 1   (wavefront)
//   D2H chunk verdicts -> host plans the per-request fallback
//   k_indiv  failed chunks' requests + non-batchable requests          (wavefront)
// All kernels of a call run on the context's stream; the host waits twice
// (chunk verdicts, final verdicts).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <sys/random.h>
#include <time.h>
#include <unistd.h>

#include <dlfcn.h>
#include <stdlib.h>
#include <zlib.h>

#include <atomic>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "bls/group_decode.hpp"
#include "launchers.hpp"

using namespace bls;

struct bls_gpu_ctx {
  int device;
  hipStream_t stream;
  hipEvent_t ev0, ev1;
  hipEvent_t ev[9];  // stage boundaries of the last verify call
  // the event the verify path polls instead of spinning in hipStreamSynchronize when
  // the call's pass is large (wait_block, pass_wait)
  hipEvent_t ev_wait;
  bool wait_block;
  char err[512];
  // device pubkey table (affine, Montgomery)
  G1A* table;
  uint32_t table_n, table_cap;
  uint32_t debug_flags;  // bls_gpu_set_debug_flags
  // the context's last pass failed its merged check: its next pass keeps the per-set
  // [r] sig chains rather than the Pippenger sum (verify_body use_msm), so a failure
  // there does not relaunch them (profiles/r05_ab_msm_min.json)
  bool last_merged_failed;
  // grow-only device workspace and pinned staging
  uint32_t* msm_state;  // MSM bucket counters + tickets (MSM_STATE_WORDS), zero between passes
  uint8_t* dev_ws;
  size_t dev_ws_cap;
  uint8_t* host_stage;      // verify inputs, pinned + device-mapped: kernels read them in place
  uint8_t* host_stage_dev;  // device view of host_stage
  size_t host_stage_cap;
  uint8_t* host_res;        // verify results written by kernels (host-mapped, coherent)
  uint8_t* host_res_dev;
  size_t host_res_cap;
  uint32_t* first_bad;      // two device slots for first_bad_pk (k_pk resets the next call's)
  uint32_t first_bad_slot;
  // cooperative programs (coop_tables.bin, tools/gen_coop.py)
  CoopEnv coop;
  void* coop_dev;
  std::vector<std::pair<std::string, CoopProg>>* coop_progs;
  // one call at a time per context: every entry point that touches the stream,
  // workspace or table holds this (callers may share a context across threads)
  std::mutex* mu;
  int admitted;  // counted by the scratch admission (bls_scratch_plan): 0 no, 1 normal, 2 high priority
};

#define CTX_LOCK(ctx) std::lock_guard<std::mutex> ctx_guard_(*(ctx)->mu)

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
  uint8_t* host = nullptr;  // offsets below `split` map into this (device view of pinned memory)
  size_t split = 0;
  template <class T>
  T* take(size_t count) {
    off = (off + 255) & ~(size_t)255;
    T* p = (T*)(base ? (off < split && host ? host : base) + off : nullptr);
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

// Pinned, device-mapped, coherent host memory: the kernels of a verify call read its
// inputs from here and write its results here, so a call moves no data with copy or
// fill blits (those queue behind other contexts' and wait for CU slots under load).
int ensure_mapped(bls_gpu_ctx* ctx, size_t bytes, uint8_t** host, uint8_t** dev, size_t* cap_io) {
  if (bytes <= *cap_io) return 0;
  if (*host) HIPC(ctx, hipHostFree(*host));
  *host = *dev = nullptr;
  size_t cap = bytes + bytes / 4 + 4096;
  HIPC(ctx, hipHostMalloc((void**)host, cap, hipHostMallocMapped | hipHostMallocCoherent));
  HIPC(ctx, hipHostGetDevicePointer((void**)dev, *host, 0));
  *cap_io = cap;
  return 0;
}

int ensure_host(bls_gpu_ctx* ctx, size_t bytes) {
  return ensure_mapped(ctx, bytes, &ctx->host_stage, &ctx->host_stage_dev, &ctx->host_stage_cap);
}

// Write a host array into the staging area behind its device-side pointer.
template <class T>
void stage_copy(bls_gpu_ctx* ctx, const T* dev_ptr, const void* src, size_t bytes) {
  if (!src || !bytes) return;
  size_t off = (const uint8_t*)dev_ptr - ctx->host_stage_dev;
  memcpy(ctx->host_stage + off, src, bytes);
}

// host view of a pointer into the result area
template <class T>
T* res_host(bls_gpu_ctx* ctx, T* dev_ptr) {
  return (T*)(ctx->host_res + ((uint8_t*)dev_ptr - ctx->host_res_dev));
}

}  // namespace

extern "C" int bls_gpu_device_count(void);
extern "C" void bls_gpu_close(bls_gpu_ctx* ctx);

// ---------------------------------------------------------------------------
// cooperative program tables: lodestar_amd/_native/coop_tables.bin next to this
// library (or $BLS_COOP_TABLES), generated by tools/gen_coop.py at build time.
// ---------------------------------------------------------------------------
namespace {

struct CoopHeader {
  char magic[4];
  uint32_t version, n_consts, n_progs, n_steps;
};
struct CoopProgEntry {
  char name[32];
  uint32_t first, n_steps, frame, n_mul;
};

// the gzip'd table (coop_tables.bin.gz, what travels with the tree) next to the
// library; $BLS_COOP_TABLES may name a plain or gzip'd file (gzread reads both)
std::string coop_tables_path() {
  const char* env = getenv("BLS_COOP_TABLES");
  if (env && *env) return env;
  Dl_info info;
  if (dladdr((void*)&bls_gpu_device_count, &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    size_t slash = p.rfind('/');
    return (slash == std::string::npos ? std::string(".") : p.substr(0, slash)) + "/coop_tables.bin.gz";
  }
  return "coop_tables.bin.gz";
}

}  // namespace

static int load_coop_tables(bls_gpu_ctx* ctx) {
  std::string path = coop_tables_path();
  gzFile f = gzopen(path.c_str(), "rb");
  if (!f) {
    snprintf(ctx->err, sizeof(ctx->err), "cannot open %s (run the build: tools/gen_coop.py)", path.c_str());
    return -1;
  }
  std::vector<uint8_t> buf;
  for (;;) {
    const size_t at = buf.size();
    buf.resize(at + (4u << 20));
    const int got = gzread(f, buf.data() + at, 4u << 20);
    if (got < 0) {
      gzclose(f);
      snprintf(ctx->err, sizeof(ctx->err), "read error in %s", path.c_str());
      return -1;
    }
    buf.resize(at + (size_t)got);
    if (got == 0) break;
  }
  gzclose(f);
  const long sz = (long)buf.size();
  const size_t got = buf.size();
  CoopHeader h;
  if (got != (size_t)sz || sz < (long)sizeof(h)) {
    snprintf(ctx->err, sizeof(ctx->err), "short read of %s", path.c_str());
    return -1;
  }
  memcpy(&h, buf.data(), sizeof(h));
  size_t consts_off = sizeof(h), progs_off = consts_off + (size_t)h.n_consts * sizeof(Fp);
  size_t steps_off = progs_off + (size_t)h.n_progs * sizeof(CoopProgEntry);
  size_t steps_bytes = (size_t)h.n_steps * COOP_LANES * sizeof(CoopOp);
  // version 4: lane groups (op kinds 3 / 4, group sizes in the step flags) and the
  // per-step term bounds (coop.hpp CoopOp)
  if (memcmp(h.magic, "BLSC", 4) != 0 || h.version != 4 || steps_off + steps_bytes != (size_t)sz) {
    snprintf(ctx->err, sizeof(ctx->err), "%s: bad coop table format", path.c_str());
    return -1;
  }
  static_assert(sizeof(CoopOp) == 80, "CoopOp layout");
  // device copy: [ops | consts | the CoopEnv struct (filled at the end)]
  size_t ops_bytes = (steps_bytes + 255) & ~(size_t)255;
  const size_t env_off = (ops_bytes + (size_t)h.n_consts * sizeof(Fp) + 255) & ~(size_t)255;
  HIPC(ctx, hipMalloc(&ctx->coop_dev, env_off + sizeof(CoopEnv)));
  uint8_t* d = (uint8_t*)ctx->coop_dev;
  HIPC(ctx, hipMemcpy(d, buf.data() + steps_off, steps_bytes, hipMemcpyHostToDevice));
  HIPC(ctx, hipMemcpy(d + ops_bytes, buf.data() + consts_off, (size_t)h.n_consts * sizeof(Fp), hipMemcpyHostToDevice));
  ctx->coop.ops = (const CoopOp*)d;
  ctx->coop.consts = (const Fp*)(d + ops_bytes);
  ctx->coop.n_consts = h.n_consts;
  if (h.n_consts > COOP_MAX_CONSTS) {
    snprintf(ctx->err, sizeof(ctx->err), "%s: %u constants > %d", path.c_str(), h.n_consts, COOP_MAX_CONSTS);
    return -1;
  }
  struct {
    const char* name;
    CoopProg* dst;
  } want[] = {{"fin_fmul", &ctx->coop.fin_fmul},         {"fin_fe1", &ctx->coop.fin_fe1},
              {"fin_fe2", &ctx->coop.fin_fe2},           {"pset_prep", &ctx->coop.pset_prep},
              {"fin_fe2_w2", &ctx->coop.fin_fe2_w2},
              {"pset_dbl_all", &ctx->coop.pset_dbl_all}, {"pset_add_x", &ctx->coop.pset_add_x},
              {"pset_phase2", &ctx->coop.pset_phase2},
              {"pset_norm2", &ctx->coop.pset_norm2},     {"pset_affine2", &ctx->coop.pset_affine2},
              {"pset_ml2", &ctx->coop.pset_ml2},         {"pset_ml2_w2", &ctx->coop.pset_ml2_w2},
              {"pset_xchain", &ctx->coop.pset_xchain},
              {"ml1_1", &ctx->coop.ml1_1},
              {"ml1_2", &ctx->coop.ml1_2}};
  ctx->coop_progs = new std::vector<std::pair<std::string, CoopProg>>();
  for (uint32_t k = 0; k < h.n_progs; ++k) {
    CoopProgEntry e;
    memcpy(&e, buf.data() + progs_off + k * sizeof(e), sizeof(e));
    e.name[31] = 0;
    ctx->coop_progs->push_back({std::string(e.name), CoopProg{e.first, e.n_steps}});
  }
  // packed programs (tools/gen_pset.py S = 2, 3): pset{S}_{prep, dbl_all, add_x, ...}
  std::vector<std::pair<std::string, CoopProg*>> want_packed;
  for (int S = 2; S <= 3; ++S) {
    CoopPsetN& pn = ctx->coop.packed[S - 2];
    const std::string pre = "pset" + std::to_string(S) + "_";
    want_packed.push_back({pre + "prep", &pn.prep});
    want_packed.push_back({pre + "dbl_all", &pn.dbl_all});
    want_packed.push_back({pre + "add_x", &pn.add_x});
    want_packed.push_back({pre + "phase2", &pn.phase2});
    want_packed.push_back({pre + "norm2", &pn.norm2});
    want_packed.push_back({pre + "affine2", &pn.affine2});
    want_packed.push_back({pre + "ml2", &pn.ml2});
  }
  for (auto& wp : want_packed) {
    bool found = false;
    for (auto& e : *ctx->coop_progs)
      if (e.first == wp.first) {
        *wp.second = e.second;
        found = true;
      }
    if (!found) {
      snprintf(ctx->err, sizeof(ctx->err), "%s: program %s missing", path.c_str(), wp.first.c_str());
      return -1;
    }
  }
  for (auto& w : want) {
    bool found = false;
    for (uint32_t k = 0; k < h.n_progs; ++k) {
      CoopProgEntry e;
      memcpy(&e, buf.data() + progs_off + k * sizeof(e), sizeof(e));
      if (strncmp(e.name, w.name, sizeof(e.name)) == 0) {
        w.dst->first = e.first;
        w.dst->n = e.n_steps;
        found = true;
      }
    }
    if (!found) {
      snprintf(ctx->err, sizeof(ctx->err), "%s: program %s missing", path.c_str(), w.name);
      return -1;
    }
  }
  // kernels take the struct by pointer (its ~370 bytes by value, next to PipeBufs, made
  // the cooperative kernels' arguments ~830 bytes)
  ctx->coop.dev = (const CoopEnv*)((uint8_t*)ctx->coop_dev + env_off);
  HIPC(ctx, hipMemcpy((void*)ctx->coop.dev, &ctx->coop, sizeof(CoopEnv), hipMemcpyHostToDevice));
  return 0;
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
// sets of the verify calls running now, over every context of the process (the Miller
// loops pick their shape by it: kernels/k_mlq.hip launch_k_mlqf)
static std::atomic<uint64_t> g_sets_in_flight{0};
uint64_t bls_sets_in_flight() { return g_sets_in_flight.load(std::memory_order_relaxed); }

// ---------------------------------------------------------------------------
// Scratch admission.  The HIP runtime backs every hardware queue with private-segment
// (scratch) memory for a full device of the deepest kernel dispatched on it, and past
// ~8 GiB over the queues in use it aborts them with HSA_STATUS_ERROR_OUT_OF_RESOURCES:
// every call in flight in the process fails and later calls too
// (profiles/r03_scratch_out_of_resources.txt; 16 queues at 464 MiB ran, 16 at 520 MiB
// and 20 at 456 MiB aborted).  So a context is admitted only while the queues its
// contexts map onto, times the deepest verify-path kernel's reservation (baked at build
// time from the kernels' resource usage, lodestar_amd/build.py), fit a budget; otherwise
// bls_gpu_init_priority returns BLS_ERR_ADMISSION with a message, as the reference's pool
// records a worker that failed to start (multithread/index.ts:221-229) and fails queued
// work only when every worker failed (:247-253).
//   queues in use: HIP maps a process's streams of one priority onto at most
//   GPU_MAX_HW_QUEUES hardware queues (default 4), per priority level.
// ---------------------------------------------------------------------------
#ifndef BLS_SCRATCH_PER_QUEUE
#define BLS_SCRATCH_PER_QUEUE 0ull  // set by lodestar_amd/build.py (-D); 0 = unknown (no limit)
#endif
#ifndef BLS_SCRATCH_WORST_KERNEL
#define BLS_SCRATCH_WORST_KERNEL "unknown"
#endif
#define BLS_SCRATCH_BUDGET_DEFAULT (6ull << 30)  // 75 % of the ~8 GiB abort point

namespace {
std::mutex g_adm_mu;
constexpr int ADM_MAX_DEV = 64;
uint32_t g_adm_normal[ADM_MAX_DEV], g_adm_high[ADM_MAX_DEV];
std::atomic<uint64_t> g_adm_budget_override{0};
thread_local char g_init_err[512];

// The HIP runtime maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues per
// priority (HIP's default 4), read once when the runtime initialises, and streams
// sharing a queue serialise: 12 contexts x 22 calls give 2.27M sets/s on 4 queues
// against 3.42M on 16 and 3.65M on 24 (bench.py hw_queues_4 / hw_queues_16,
// profiles/r05_bench_first.json).  The library never writes the environment by itself
// (a load-time setenv would race getenv on a multithreaded host's other threads and leak
// into every child process): the host asks with bls_gpu_request_hw_queues before any
// HIP use (the Python and JS wrappers do as they load the library), and the library
// records what the runtime really got -- the variable's value when the runtime
// initialised, if that happened under this library's first context, or "unknown" when
// another component of the process had initialised HIP first (hw_queues_known = 0 in
// bls_admission, and one warning on stderr when the runtime then most likely kept
// HIP's 4 queues).
namespace {
// the render / KFD device is open once the ROCm runtime initialised in this process
bool hip_runtime_up() {
  char path[64], target[64];
  for (int fd = 0; fd < 4096; ++fd) {
    snprintf(path, sizeof(path), "/proc/self/fd/%d", fd);
    const ssize_t n = readlink(path, target, sizeof(target) - 1);
    if (n <= 0) continue;
    target[n] = 0;
    if (strcmp(target, "/dev/kfd") == 0) return true;
  }
  return false;
}

uint32_t parse_hwq(const char* e) {
  const long v = e && *e ? strtol(e, nullptr, 10) : 0;
  return v > 0 ? (uint32_t)v : 4u;
}

bool g_hip_up_at_load = false;  // HIP was initialised before this library loaded
// the runtime's queue count: fixed at this library's first context (when the runtime
// came up under it, hwq_known = 1) or guessed from the environment (hwq_known = 0)
std::once_flag g_hwq_once;
uint32_t g_hwq_effective = 0;
bool g_hwq_known = false;

__attribute__((constructor)) void bls_record_runtime_state() { g_hip_up_at_load = hip_runtime_up(); }

// called by bls_gpu_init_priority before its first HIP call (g_adm_mu held)
void note_runtime_queues() {
  std::call_once(g_hwq_once, [] {
    const bool up = g_hip_up_at_load || hip_runtime_up();
    const char* e = getenv("GPU_MAX_HW_QUEUES");
    g_hwq_effective = parse_hwq(e);
    g_hwq_known = !up;
    if (up && !(e && *e))
      fprintf(stderr,
              "lodestar_bls: warning: the HIP runtime was initialised before this library's first context, "
              "with GPU_MAX_HW_QUEUES unset: its streams share HIP's default 4 hardware queues per priority, so "
              "more than 4 verifier contexts serialise (set GPU_MAX_HW_QUEUES before the process's first HIP "
              "call, or call bls_gpu_request_hw_queues first; INTEGRATION.md section 4)\n");
  });
}
}  // namespace

uint32_t hw_queues_env() {
  if (g_hwq_effective) return g_hwq_effective;
  return parse_hwq(getenv("GPU_MAX_HW_QUEUES"));
}

uint64_t scratch_budget() {
  const uint64_t o = g_adm_budget_override.load();
  if (o) return o;
  const char* e = getenv("BLS_SCRATCH_BUDGET_MIB");
  const unsigned long long v = e && *e ? strtoull(e, nullptr, 10) : 0ull;
  return v ? (uint64_t)v << 20 : BLS_SCRATCH_BUDGET_DEFAULT;
}

void init_fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void init_fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_init_err, sizeof(g_init_err), fmt, ap);
  va_end(ap);
}
}  // namespace

extern "C" {

int bls_scratch_plan(uint32_t n_normal, uint32_t n_high, uint32_t hw_queues, bls_admission* out) {
  bls_admission a;
  memset(&a, 0, sizeof(a));
  a.contexts_normal = n_normal;
  a.contexts_high = n_high;
  a.hw_queues = hw_queues ? hw_queues : hw_queues_env();
  a.hw_queues_known = hw_queues ? 1u : (g_hwq_effective ? (g_hwq_known ? 1u : 0u) : 2u);
  a.queues_in_use = (n_normal < a.hw_queues ? n_normal : a.hw_queues) + (n_high < a.hw_queues ? n_high : a.hw_queues);
  a.scratch_per_queue = BLS_SCRATCH_PER_QUEUE;
  a.scratch_reserved = (uint64_t)a.queues_in_use * a.scratch_per_queue;
  a.scratch_budget = scratch_budget();
  if (out) *out = a;
  return a.scratch_reserved <= a.scratch_budget ? 0 : BLS_ERR_ADMISSION;
}

const char* bls_scratch_worst_kernel(void) { return BLS_SCRATCH_WORST_KERNEL; }

int bls_gpu_request_hw_queues(uint32_t n) {
  if (n == 0) return -2;
  const char* e = getenv("GPU_MAX_HW_QUEUES");
  if (e && *e) return 1;  // the host's own choice stands
  if (g_hip_up_at_load || g_hwq_effective || hip_runtime_up()) return 2;  // too late: the runtime has its count
  char v[16];
  snprintf(v, sizeof(v), "%u", n);
  return setenv("GPU_MAX_HW_QUEUES", v, 0) == 0 ? 0 : -1;
}

int bls_gpu_admission(int device, bls_admission* out) {
  if (device < 0 || device >= ADM_MAX_DEV) return -2;
  std::lock_guard<std::mutex> g(g_adm_mu);
  return bls_scratch_plan(g_adm_normal[device], g_adm_high[device], 0, out);
}

void bls_gpu_set_scratch_budget(uint64_t bytes) { g_adm_budget_override.store(bytes); }

const char* bls_gpu_init_error(void) { return g_init_err; }

int bls_gpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int bls_gpu_init(int device, bls_gpu_ctx** out) { return bls_gpu_init_priority(device, BLS_PRIORITY_NORMAL, out); }

int bls_gpu_init_priority(int device, int priority, bls_gpu_ctx** out) {
  if (!out) return -2;
  *out = nullptr;
  g_init_err[0] = 0;
  if (device < 0 || device >= ADM_MAX_DEV) {
    init_fail("bls_gpu_init: device %d out of range", device);
    return -2;
  }
  const bool high = priority == BLS_PRIORITY_HIGH;
  {
    // admit first: a refused context never creates its stream (no queue, no reservation)
    std::lock_guard<std::mutex> g(g_adm_mu);
    note_runtime_queues();  // before this library's first HIP call
    bls_admission a;
    const uint32_t nn = g_adm_normal[device] + (high ? 0u : 1u), nh = g_adm_high[device] + (high ? 1u : 0u);
    if (bls_scratch_plan(nn, nh, 0, &a) != 0) {
      init_fail("BLS_ERR_ADMISSION: a %s-priority context on device %d would map %u normal + %u high-priority "
                "contexts onto %u hardware queues (GPU_MAX_HW_QUEUES=%u), reserving %llu MiB of scratch "
                "(%llu MiB per queue for %s) > the %llu MiB budget ($BLS_SCRATCH_BUDGET_MIB); close a context or "
                "lower the context count",
                high ? "high" : "normal", device, nn, nh, a.queues_in_use, a.hw_queues,
                (unsigned long long)(a.scratch_reserved >> 20), (unsigned long long)(a.scratch_per_queue >> 20),
                BLS_SCRATCH_WORST_KERNEL, (unsigned long long)(a.scratch_budget >> 20));
      return BLS_ERR_ADMISSION;
    }
    if (high) ++g_adm_high[device];
    else ++g_adm_normal[device];
  }
  bls_gpu_ctx* ctx = new bls_gpu_ctx();
  memset(ctx, 0, sizeof(*ctx));
  ctx->mu = new std::mutex();
  ctx->device = device;
  ctx->admitted = high ? 2 : 1;
  // every failure below releases what was made through bls_gpu_close (it tolerates
  // members that were never created) and leaves its message for bls_gpu_init_error
  auto fail = [&](const char* what, hipError_t e) {
    init_fail("bls_gpu_init: %s: %s", what, hipGetErrorString(e));
    bls_gpu_close(ctx);
    return -1;
  };
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return fail("hipSetDevice", e);
  int prio_lo = 0, prio_hi = 0;  // HIP: numerically lower = higher priority
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if ((e = hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, high ? prio_hi : prio_lo)) != hipSuccess)
    return fail("hipStreamCreateWithPriority", e);
  if ((e = hipEventCreate(&ctx->ev0)) != hipSuccess || (e = hipEventCreate(&ctx->ev1)) != hipSuccess)
    return fail("hipEventCreate", e);
  for (int i = 0; i < 9; ++i)
    if ((e = hipEventCreate(&ctx->ev[i])) != hipSuccess) return fail("hipEventCreate", e);
  if ((e = hipEventCreateWithFlags(&ctx->ev_wait, hipEventDisableTiming)) != hipSuccess)
    return fail("hipEventCreateWithFlags", e);
  if (load_coop_tables(ctx) != 0) {
    init_fail("bls_gpu_init: %s", ctx->err);
    bls_gpu_close(ctx);
    return -1;
  }
  if ((e = hipMalloc(&ctx->first_bad, 2 * sizeof(uint32_t))) != hipSuccess ||
      (e = hipMemset(ctx->first_bad, 0xFF, 2 * sizeof(uint32_t))) != hipSuccess)
    return fail("first_bad", e);
  // the MSM's bucket counters and tickets: zeroed here once, then reset by the kernels'
  // last workgroups (and re-zeroed after a failed call, verify_impl)
  if ((e = hipMalloc(&ctx->msm_state, sizeof(uint32_t) * MSM_STATE_WORDS)) != hipSuccess ||
      (e = hipMemset(ctx->msm_state, 0, sizeof(uint32_t) * MSM_STATE_WORDS)) != hipSuccess)
    return fail("msm_state", e);
  *out = ctx;
  return 0;
}

void bls_gpu_close(bls_gpu_ctx* ctx) {
  if (!ctx) return;
  ctx->mu->lock();  // wait for a call in flight on another thread
  ctx->mu->unlock();
  if (ctx->admitted) {
    std::lock_guard<std::mutex> g(g_adm_mu);
    if (ctx->admitted == 2) --g_adm_high[ctx->device];
    else --g_adm_normal[ctx->device];
    ctx->admitted = 0;
  }
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->table) (void)hipFree(ctx->table);
  if (ctx->dev_ws) (void)hipFree(ctx->dev_ws);
  if (ctx->host_stage) (void)hipHostFree(ctx->host_stage);
  if (ctx->host_res) (void)hipHostFree(ctx->host_res);
  if (ctx->first_bad) (void)hipFree(ctx->first_bad);
  if (ctx->msm_state) (void)hipFree(ctx->msm_state);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->ev_wait) (void)hipEventDestroy(ctx->ev_wait);
  for (int i = 0; i < 9; ++i)
    if (ctx->ev[i]) (void)hipEventDestroy(ctx->ev[i]);
  if (ctx->coop_dev) (void)hipFree(ctx->coop_dev);
  delete ctx->coop_progs;
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx->mu;
  delete ctx;
}

const char* bls_gpu_last_error(const bls_gpu_ctx* ctx) { return ctx ? ctx->err : "no context"; }

int64_t bls_gpu_load_pubkeys(bls_gpu_ctx* ctx, const uint8_t* pks, uint32_t n, uint32_t pk_len, int32_t* codes) {
  CTX_LOCK(ctx);
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
  std::vector<int32_t> host_codes(n);
  HIPC(ctx, hipMemcpyAsync(host_codes.data(), d_codes, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  if (codes) memcpy(codes, host_codes.data(), sizeof(int32_t) * n);
  // all or nothing: a key that does not decode leaves the table as it was, so table
  // indices (validator indices) stay aligned across contexts and calls
  for (uint32_t i = 0; i < n; ++i)
    if (host_codes[i] != 0) return ctx->table_n;
  ctx->table_n += n;
  return ctx->table_n;
}

int bls_gpu_validate_pubkeys(bls_gpu_ctx* ctx, const uint8_t* pks, uint32_t n, uint32_t pk_len, int32_t* codes) {
  CTX_LOCK(ctx);
  if ((pk_len != 48 && pk_len != 96) || !codes) {
    snprintf(ctx->err, sizeof(ctx->err), "pk_len must be 48 or 96 and codes non-null");
    return -2;
  }
  if (n == 0) return 0;
  HIPC(ctx, hipSetDevice(ctx->device));
  const size_t in_bytes = (size_t)pk_len * n;
  Carver cv{nullptr, 0};
  cv.take<uint8_t>(in_bytes);
  cv.take<int32_t>(n);
  if (ensure_dev(ctx, cv.off)) return -1;
  Carver c2{ctx->dev_ws, 0};
  uint8_t* d_in = c2.take<uint8_t>(in_bytes);
  int32_t* d_codes = c2.take<int32_t>(n);
  HIPC(ctx, hipMemcpyAsync(d_in, pks, in_bytes, hipMemcpyHostToDevice, ctx->stream));
  HIPC(ctx, launch_k_validate_pubkeys(d_in, n, pk_len, d_codes, ctx->stream));
  HIPC(ctx, hipMemcpyAsync(codes, d_codes, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

// One verifyManySignatureSets call (partial_out == nullptr), or the Miller-loop
// partial of one shard of a sharded call (bls_gpu_partial): the same front half
// (decode, hash_to_G2, per-set programs, exact path, status), then either the
// chunk / individual verdicts or a product tree of every f_i.
// Aggregated-signature path (k_chain + k_gsum + k_vset + k_mln single-pair Miller
// loops, one signature Miller loop per chunk) from SIGAGG_MIN_SETS sets on, except for
// calls of at most PERSET_MAX_CALL sets while the process has at most
// $BLS_PERSET_MAX_INFLIGHT (20,480) sets in flight (this call's included): those run the
// all-cooperative k_pset / k_psetn (a set's chains spread over a wavefront instead of one
// lane: shorter calls while the device has room, fewer sets per second once it is full --
// per-set vs aggregated at 12 x 1024-set calls in flight 0.82M vs 0.56M sets/s, 16 x 1024
// 0.82M vs 0.72M, 24 x 1024 1.02M vs 1.03M, profiles/r04_ab_perset_crossover.json).  A call of more sets would fill
// every SIMD with its wavefronts (2 sets each, two per SIMD) and hold the main-thread
// lane's context behind it (test_napi.py: a 4096-set pool call finished first).
// BLS_DEBUG_SIGAGG_ON / _OFF or $BLS_SIGAGG (0 / 1) force a path.
#define SIGAGG_MIN_SETS 512u
#define PERSET_MAX_CALL 2048u
static bool use_sigagg(const bls_gpu_ctx* ctx, uint32_t n) {
  static const int env = [] {
    const char* e = getenv("BLS_SIGAGG");
    return e ? atoi(e) : -1;
  }();
  static const uint64_t perset_max = [] {
    const char* e = getenv("BLS_PERSET_MAX_INFLIGHT");
    return e ? (uint64_t)strtoull(e, nullptr, 10) : 20480ull;
  }();
  if (ctx->debug_flags & BLS_DEBUG_SIGAGG_ON) return true;
  if (ctx->debug_flags & BLS_DEBUG_SIGAGG_OFF) return false;
  if (env >= 0) return env != 0;
  return n >= SIGAGG_MIN_SETS && (n > PERSET_MAX_CALL || bls_sets_in_flight() > perset_max);
}

// $BLS_DEBUG_SYNC: synchronise after every kernel of a verify call and log its name
// and wall time to stderr (a kernel that never finishes is the last name printed)
static void dbg_sync(hipStream_t s, const char* what) {
  static const bool on = getenv("BLS_DEBUG_SYNC") != nullptr;
  if (!on) return;
  timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  fprintf(stderr, "[bls sync] %s ...", what);
  fflush(stderr);
  hipError_t e = hipStreamSynchronize(s);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  fprintf(stderr, " %.3f ms %s\n", (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) * 1e-6,
          hipGetErrorString(e));
  fflush(stderr);
}

// Group testing of a failed chunk's requests (instead of one final exponentiation per
// request, worker.ts:91-98).  Each request's product F_t (its sets' f and, on the
// aggregated path, its own signature-sum pairing) is left by k_indiv_coop; a test is
// FE(prod of a group's F_t) == 1 (k_group_coop), the same random-scalar batch check the
// reference runs over a chunk.  With the chunk's requests of status OK indexed 0 .. m-1:
//   pass A: the group of all of them (A), and for each bit j of the index the group G_j
//           of those with bit j set; each G_j's final exponentiation is also compared with
//           A's (k_group_cmp): FE(G_j) FE(rest_j) = FE(A), so FE(rest_j) == 1 iff
//           FE(G_j) == FE(A) -- every test answers for its complement too;
//   a single invalid request b fails exactly one of G_j, rest_j for every j (G_j where
//   b's bit j is set), which names b, and every other request sits in a passing test;
//   pass C: any other outcome (both of some G_j, rest_j failing: two or more invalid; an
//           index past m): every request alone.
// With one invalid request in a chunk of 16 that is 5 final exponentiations in one round
// instead of 16 (round 6; before it, without the comparison, pass B tested {b} alone and
// the rest together: 6 in two rounds, $BLS_GROUP_EQ=0 restores that); verdicts and the worker counters are the reference's (a test that passes is the
// batch the reference's retry would have passed request by request, with the same
// soundness).  On for chunks of >= 4 requests since round 6: once the failed chunks'
// requests stopped re-running their sets' own Miller loops and the chunks of a failing
// stream are checked without the merged check first, the saved final exponentiations
// outweigh the extra rounds -- cfg4 per-set requests 1.35M -> 1.50M sets/s steady, cfg5
// level (profiles/r06_ab_group_test.json; in rounds 4-5 it lost or was level,
// r04_ab_group_test.json, r05_ab_group_test_again.json).  $BLS_GROUP_TEST_MIN sets the
// smallest chunk tested so (0 = off); BLS_DEBUG_GROUP_TEST forces chunks of >= 4.
static uint32_t group_test_min(const bls_gpu_ctx* ctx) {
  static const uint32_t v = [] {
    const char* e = getenv("BLS_GROUP_TEST_MIN");
    const long x = e ? atol(e) : 4;
    return x <= 0 ? 0xFFFFFFFFu : (uint32_t)(x < 2 ? 2 : x);
  }();
  return (ctx->debug_flags & BLS_DEBUG_GROUP_TEST) ? 4u : v;
}

// Group sums (aggregated path): the tests' own signature sums, sum of r_i sig_i over
// their requests' sets, paired ML(-g1, .) into sum_f[g] before k_group_coop; returns 0,
// 1 when the plan does not fit the workspace (the caller tests the requests alone), < 0
// on an error.  Unset: each request's product already holds its own sum's pairing.
typedef std::function<int(const std::vector<uint32_t>&, const std::vector<uint32_t>&)> GroupSums;

// group sums (run_group_tests) for a pass with at least $BLS_GROUP_SUMS_MIN (512)
// group-tested requests; 0 = always, $BLS_GROUP_SUMS=0 = never.  They save Miller loops
// (cfg4 per-set requests, ~1,300 group-tested requests a pass: 1.52M -> 1.56M sets/s
// steady) but put a sum + Miller-loop stage in front of each round of tests, where the
// per-request sums ride in the requests' Miller-loop launch: with a few failed chunks
// a pass (the cfg5 slice, ~80 requests) that latency costs more (3.29M -> 3.05M)
// (profiles/r06_ab_group_sums.json)
static bool group_sums_on(size_t n_group_tested) {
  static const bool on = [] {
    const char* e = getenv("BLS_GROUP_SUMS");
    return !(e && atoi(e) == 0);
  }();
  static const size_t min_reqs = [] {
    const char* e = getenv("BLS_GROUP_SUMS_MIN");
    return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)512;
  }();
  return on && n_group_tested >= min_reqs;
}

// complement inference in the group tests (verify_groups): pass A carries each chunk's
// test of all its requests and compares the bit groups' final exponentiations with it, so
// one invalid request is found without pass B ({b} alone, the rest together); the whole's
// value is the failed chunk check's own final exponentiation where that ran over the same
// requests (k_chunk_coop keeps it in b.chunk_fe), else a test of them.  $BLS_GROUP_EQ=0
// restores the two rounds, =2 always tests the whole
static int group_eq_mode() {
  static const int mode = [] {
    const char* e = getenv("BLS_GROUP_EQ");
    return e ? atoi(e) : 1;
  }();
  return mode;
}
static bool group_eq_on() { return group_eq_mode() != 0; }

// run the tests (goff: offsets into gmem, indices into the indiv list); results in gv
// (bit 0: passed; bit 1, with ref: its final exponentiation equals test ref[g]'s);
// 1 when the group sums do not fit (nothing ran)
static hipError_t pass_wait(bls_gpu_ctx* ctx, hipStream_t s);  // below, before verify_body

static int run_group_tests(bls_gpu_ctx* ctx, const PipeBufs& b, GroupBufs& g, const std::vector<uint32_t>& goff,
                           const std::vector<uint32_t>& gmem, std::vector<int32_t>& gv, hipStream_t s,
                           const GroupSums* sums, const std::vector<uint32_t>* ref = nullptr) {
  gv.assign(goff.size() - 1, 0);
  if (gv.empty()) return 0;
  if (sums && *sums) {
    const int rc = (*sums)(goff, gmem);
    if (rc != 0) return rc;
  }
  stage_copy(ctx, g.off, goff.data(), sizeof(uint32_t) * goff.size());  // the stream is idle
  stage_copy(ctx, g.members, gmem.data(), sizeof(uint32_t) * gmem.size());
  g.n = (uint32_t)gv.size();
  GroupBufs gg = g;
  if (ref) stage_copy(ctx, g.ref, ref->data(), sizeof(uint32_t) * ref->size());
  else gg.fe = nullptr;
  HIPC(ctx, launch_k_group_coop(b, ctx->coop, gg, s)); dbg_sync(s, "k_group_coop");
  HIPC(ctx, pass_wait(ctx, s));
  memcpy(gv.data(), res_host(ctx, g.verdict), sizeof(int32_t) * gv.size());
  return 0;
}

struct GtChunk {
  uint32_t beg, end;  // its requests in the indiv list
  uint32_t ch;        // its chunk (b.chunk_fe)
};

static int verify_groups(bls_gpu_ctx* ctx, const PipeBufs& b, GroupBufs& gbufs, const std::vector<GtChunk>& chunks,
                         std::vector<int32_t>& verdict, hipStream_t s, size_t grp_cap, size_t grp_mem_cap,
                         const GroupSums* sums) {
  struct Chunk {
    std::vector<uint32_t> ok;  // indiv indices of the requests of status OK
    bool has_err = false;
    bool whole = false;        // a test of all of ok at `first` (else the chunk check's value)
    uint32_t first = 0, nbits = 0;
    int32_t b = -1;            // the one invalid request's position in ok (pass B), -1 none
  };
  std::vector<Chunk> cs;
  std::vector<uint32_t> goff{0}, gmem, ref;
  const bool eq = group_eq_on() && gbufs.fe;
  auto add_test = [&](const std::vector<uint32_t>& m, uint32_t r) {
    gmem.insert(gmem.end(), m.begin(), m.end());
    goff.push_back((uint32_t)gmem.size());
    ref.push_back(r);
  };
  for (const auto& ch : chunks) {
    Chunk c;
    for (uint32_t t = ch.beg; t < ch.end; ++t) {
      if (verdict[t] == 2) c.ok.push_back(t);
      else c.has_err = true;  // its -code stays
    }
    if (c.ok.empty()) continue;
    c.first = (uint32_t)goff.size() - 1;
    // the whole's value: the failed chunk check's own final exponentiation when it ran
    // over exactly these requests (no erroneous one), else a test of them
    const bool from_check = eq && group_eq_mode() != 2 && gbufs.ref_fe && !c.has_err && c.ok.size() > 1;
    c.whole = !from_check && (eq || c.has_err || c.ok.size() == 1);
    if (c.whole) add_test(c.ok, REF_NONE);
    const uint32_t m = (uint32_t)c.ok.size();
    while (m > 1 && (1u << c.nbits) < m) ++c.nbits;
    for (uint32_t j = 0; j < c.nbits; ++j) {
      std::vector<uint32_t> g;
      for (uint32_t k = 0; k < m; ++k)
        if ((k >> j) & 1u) g.push_back(c.ok[k]);
      add_test(g, from_check ? (REF_CHUNK | ch.ch) : c.first);
    }
    cs.push_back(std::move(c));
  }
  if (gmem.size() > grp_mem_cap || goff.size() - 1 > grp_cap) {
    snprintf(ctx->err, sizeof(ctx->err), "group-test plan exceeds its workspace");
    return -3;
  }
  std::vector<int32_t> gv;
  std::vector<uint32_t> goff_b{0}, gmem_b, alone;  // alone: requests for pass C
  std::vector<size_t> in_b;
  const int rc_a = run_group_tests(ctx, b, gbufs, goff, gmem, gv, s, sums, eq ? &ref : nullptr);
  if (rc_a < 0) return -1;
  if (rc_a == 1) {  // the group sums of pass A do not fit: every request alone
    for (const Chunk& c : cs) alone.insert(alone.end(), c.ok.begin(), c.ok.end());
    cs.clear();
  }
  // complement inference: with the test of all the chunk's requests (A) beside each bit
  // group G_j, FE(G_j) FE(rest_j) = FE(A) decides the complement too (FE(rest_j) == 1 iff
  // FE(G_j) == FE(A)), so a single invalid request b shows as exactly one failing test per
  // bit -- G_j where b's bit j is set, rest_j where it is clear -- and every other request
  // sits in a passing test: no pass B.  Both G_j and rest_j failing (two or more invalid)
  // or an index past m: pass C.
  for (size_t i = 0; eq && i < cs.size(); ++i) {
    const Chunk& c = cs[i];
    const uint32_t m = (uint32_t)c.ok.size();
    // without a whole test the whole is the failed chunk check (it failed)
    const bool pass = c.whole && (gv[c.first] & 1) != 0;
    const int32_t bad = group_decode(m, c.nbits, pass, gv.data() + c.first + (c.whole ? 1u : 0u));
    if (bad < 0) {
      alone.insert(alone.end(), c.ok.begin(), c.ok.end());
      continue;
    }
    for (uint32_t k = 0; k < m; ++k) verdict[c.ok[k]] = (int32_t)k == bad ? 0 : 1;
  }
  if (eq) cs.clear();
  // decode pass A; plan pass B
  for (size_t i = 0; i < cs.size(); ++i) {
    Chunk& c = cs[i];
    uint32_t idx = c.first;
    const uint32_t m = (uint32_t)c.ok.size();
    if (c.has_err || m == 1) {
      const bool pass = gv[idx++] == 1;
      if (pass || m == 1) {
        for (uint32_t t : c.ok) verdict[t] = pass ? 1 : 0;
        continue;
      }
    }
    uint32_t bad = 0;
    for (uint32_t j = 0; j < c.nbits; ++j)
      if (gv[idx + j] != 1) bad |= 1u << j;
    if (bad >= m) {
      alone.insert(alone.end(), c.ok.begin(), c.ok.end());
      continue;
    }
    c.b = (int32_t)bad;
    gmem_b.push_back(c.ok[bad]);
    goff_b.push_back((uint32_t)gmem_b.size());
    for (uint32_t k = 0; k < m; ++k)
      if (k != bad) gmem_b.push_back(c.ok[k]);
    goff_b.push_back((uint32_t)gmem_b.size());
    in_b.push_back(i);
  }
  const int rc_b = in_b.empty() ? 0 : run_group_tests(ctx, b, gbufs, goff_b, gmem_b, gv, s, sums);
  if (rc_b < 0) return -1;
  for (size_t q = 0; q < in_b.size(); ++q) {
    Chunk& c = cs[in_b[q]];
    if (rc_b == 0 && gv[2 * q] == 0 && gv[2 * q + 1] == 1) {
      for (uint32_t k = 0; k < c.ok.size(); ++k) verdict[c.ok[k]] = (int32_t)k == c.b ? 0 : 1;
    } else {
      alone.insert(alone.end(), c.ok.begin(), c.ok.end());
    }
  }
  // pass C: one test per request
  std::vector<uint32_t> goff_c{0};
  for (size_t k = 0; k < alone.size(); ++k) goff_c.push_back((uint32_t)k + 1);
  const int rc_c = run_group_tests(ctx, b, gbufs, goff_c, alone, gv, s, sums);
  if (rc_c != 0) {
    // one request per test always fits the request-sum workspace
    snprintf(ctx->err, sizeof(ctx->err), "group tests: per-request sums do not fit");
    return -3;
  }
  for (size_t k = 0; k < alone.size(); ++k) verdict[alone[k]] = gv[k] == 1 ? 1 : 0;
  return 0;
}


// Pippenger merged signature sum (k_msm) instead of the per-set [r] sig chains (k_chain
// role 2, ~1.6k Fp products per set) and the k_gsum levels: ~10 % fewer instructions per
// set, but its serial stages (segments, buckets, the windows' dependent additions) make
// the pass ~5 ms longer.  So it pays only when the device is VALU-bound with many sets in
// flight: 3.46M vs 3.21M sets/s at 16 x 16, level at 12 x 16, 1.89M vs 2.25M at 4 x 16
// (profiles/r03_ab_msm.json, round 3).  On the round-5 build it is level at 4 x 16 and
// ahead from 6 x 16 on (8 x 16: 3.24M / 3.30M vs 3.00M, profiles/r05_ab_msm_min.json), so
// by default on while the process has more than $BLS_MSM_MIN (60,000) sets in flight and
// the context's last pass passed its merged check (a failing pass needs the per-set chains
// after all: relaunching them cost the epoch slice with invalid sets 2.42M -> 2.1M sets/s);
// $BLS_MSM=1 / 0 forces it on / off.
static bool msm_on() {
  static const int forced = [] {
    const char* e = getenv("BLS_MSM");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
  }();
  static const uint64_t min_sets = [] {
    const char* e = getenv("BLS_MSM_MIN");
    return e ? (uint64_t)strtoull(e, nullptr, 10) : 60000ull;
  }();
  if (forced >= 0) return forced == 1;
  return bls_sets_in_flight() > min_sets;
}

// Shared Miller loops in k_mln (PipeBufs::ml_dom): on unless $BLS_ML_SHARED=0
static bool ml_shared_on() {
  static const bool on = [] {
    const char* e = getenv("BLS_ML_SHARED");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// Merged signature sum (with the merged check): one signature Miller loop per device
// pass instead of one per chunk; on unless $BLS_SIG_TOTAL=0
static bool sig_total_on() {
  static const bool on = [] {
    const char* e = getenv("BLS_SIG_TOTAL");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// After a pass whose merged check failed, a context's next pass skips it and checks its
// chunks straight away (each chunk's own signature sum paired in the pass's Miller-loop
// launch, then the per-chunk final exponentiations): a stream with invalid sets in most
// passes (the cfg4 per-set requests, the cfg5 epoch slice) otherwise pays the merged
// final exponentiation, then the chunk sums, their Miller loops and the chunk checks one
// after another on the failing call's path.  The first pass whose chunks all pass turns
// the merged check back on.  $BLS_MERGED_AFTER_FAIL=1 keeps it on every pass.
static bool merged_skip_after_fail() {
  static const bool on = [] {
    const char* e = getenv("BLS_MERGED_AFTER_FAIL");
    return !(e && atoi(e) == 1);
  }();
  return on;
}

// Segmented-sum plan for k_gsum over groups of requests: the groups' set indices
// (group-major) and, per level, (beg, end) segments of at most GSUM_FAN items that
// never straddle a group; level 0 indexes gsets, level L > 0 the outputs of level
// L - 1.  After the last level there is one point per group, in group order.
struct GsumPlan {
  std::vector<uint32_t> gsets;
  std::vector<uint32_t> seg;        // every level's pairs, concatenated
  std::vector<uint32_t> level_off;  // level L: pairs [level_off[L], level_off[L + 1])
};

// groups given as explicit set lists: group g = sets[goff[g] .. goff[g + 1])
static void plan_gsum_sets(const std::vector<uint32_t>& goff, const std::vector<uint32_t>& sets, GsumPlan& p) {
  p.gsets = sets;
  p.seg.clear();
  p.level_off.assign(1, 0);
  const size_t G = goff.size() - 1;
  std::vector<uint32_t> cnt(G);
  for (size_t g = 0; g < G; ++g) {
    const uint32_t gb = goff[g], ge = goff[g + 1];
    cnt[g] = 0;
    for (uint32_t k = gb; k < ge || (k == gb && gb == ge); k += GSUM_FAN) {
      p.seg.push_back(k);
      p.seg.push_back(k + GSUM_FAN < ge ? k + GSUM_FAN : ge);
      ++cnt[g];
      if (gb == ge) break;
    }
  }
  p.level_off.push_back((uint32_t)(p.seg.size() / 2));
  for (;;) {
    bool more = false;
    for (uint32_t c : cnt) more = more || c > 1;
    if (!more) break;
    uint32_t pos = 0;
    for (size_t g = 0; g < G; ++g) {
      const uint32_t c = cnt[g];
      uint32_t nc = 0;
      for (uint32_t k = 0; k < c; k += GSUM_FAN, ++nc) {
        p.seg.push_back(pos + k);
        p.seg.push_back(pos + (k + GSUM_FAN < c ? k + GSUM_FAN : c));
      }
      pos += c;
      cnt[g] = nc;
    }
    p.level_off.push_back((uint32_t)(p.seg.size() / 2));
  }
}

// groups of requests (chunks, individually verified requests): their sets in order
static void plan_gsum(const bls_batch* in, const std::vector<uint32_t>& grp_off, const std::vector<uint32_t>& grp_reqs,
                      GsumPlan& p) {
  std::vector<uint32_t> goff(1, 0), sets;
  for (size_t g = 0; g + 1 < grp_off.size(); ++g) {
    for (uint32_t k = grp_off[g]; k < grp_off[g + 1]; ++k) {
      const uint32_t r = grp_reqs[k];
      for (uint32_t i = in->req_set_offsets[r]; i < in->req_set_offsets[r + 1]; ++i) sets.push_back(i);
    }
    goff.push_back((uint32_t)sets.size());
  }
  plan_gsum_sets(goff, sets, p);
}

// Miller-loop units (sum r_i pk_i per root): within each chunk, the sets
// signing the same root (msg_rep: the root's first set) form one unit, paired once as
// ML(sum r_i pk_i, H(root)).  Used when it at least halves the chunks' Miller loops.
struct UnitPlan {
  std::vector<uint32_t> set_unit, unit_rep, unit_off, goff, members;
  uint32_t n_units = 0;
};

static bool plan_units(const bls_batch* in, const BatchPlan& plan, const std::vector<uint32_t>& msg_rep, uint32_t n,
                       UnitPlan& u) {
  const uint32_t C = (uint32_t)plan.chunk_off.size() - 1;
  if (msg_rep.empty() || C == 0) return false;
  u.set_unit.assign(n, UNIT_NONE);
  u.unit_off.assign(1, 0);
  std::vector<uint32_t> stamp(n, 0xFFFFFFFFu), unit_of(n, 0);
  std::vector<std::vector<uint32_t>> mem;
  uint32_t in_chunks = 0;
  for (uint32_t c = 0; c < C; ++c) {
    for (uint32_t k = plan.chunk_off[c]; k < plan.chunk_off[c + 1]; ++k) {
      const uint32_t r = plan.chunk_reqs[k];
      for (uint32_t i = in->req_set_offsets[r]; i < in->req_set_offsets[r + 1]; ++i) {
        const uint32_t rep = msg_rep[i];
        if (stamp[rep] != c) {
          stamp[rep] = c;
          unit_of[rep] = (uint32_t)mem.size();
          mem.emplace_back();
          u.unit_rep.push_back(rep);
        }
        u.set_unit[i] = unit_of[rep];
        mem[unit_of[rep]].push_back(i);
        ++in_chunks;
      }
    }
    u.unit_off.push_back((uint32_t)mem.size());
  }
  u.n_units = (uint32_t)mem.size();
  if (2ull * u.n_units > in_chunks) return false;
  u.goff.assign(1, 0);
  u.members.clear();
  for (auto& m : mem) {
    u.members.insert(u.members.end(), m.begin(), m.end());
    u.goff.push_back((uint32_t)u.members.size());
  }
  return true;
}

// Launch the levels of `p` (seg: its pairs on the device) and k_vset for groups
// [vbase, vbase + G); tmp: two point buffers of level-0 size.
static int launch_gsum(bls_gpu_ctx* ctx, PipeBufs& b, const GsumPlan& p, const uint32_t* seg_dev,
                       const uint32_t* gsets_dev, G2J* const tmp[2], uint32_t vbase, hipStream_t s) {
  b.gsets = gsets_dev;
  const size_t levels = p.level_off.size() - 1;
  const G2J* in = nullptr;
  for (size_t L = 0; L < levels; ++L) {
    const uint32_t beg = p.level_off[L], n_seg = p.level_off[L + 1] - beg;
    HIPC(ctx, launch_k_gsum(b, seg_dev + 2 * beg, n_seg, in, tmp[L & 1], s)); dbg_sync(s, "k_gsum");
    in = tmp[L & 1];
  }
  const uint32_t G = levels ? p.level_off[levels] - p.level_off[levels - 1] : 0;
  HIPC(ctx, launch_k_vset(b, in, G, vbase, s)); dbg_sync(s, "k_vset");
  return 0;
}

// plan_batch over several worker messages submitted together (bls_gpu_verify_many):
// each message's batchable requests are chunked on their own (worker.ts:56 runs per
// message), so the chunks never straddle a message; req_bounds[k] = first request of
// message k, req_bounds[n_msgs] = n_reqs.
static void plan_batch_msgs(const bls_batch* in, const std::vector<uint32_t>& req_bounds, BatchPlan& p) {
  p.chunk_off.assign(1, 0);
  p.chunk_reqs.clear();
  p.nonbatch_reqs.clear();
  std::vector<uint32_t> batchable, bounds;
  for (size_t m = 0; m + 1 < req_bounds.size(); ++m) {
    batchable.clear();
    for (uint32_t r = req_bounds[m]; r < req_bounds[m + 1]; ++r) {
      if (in->req_batchable && in->req_batchable[r]) batchable.push_back(r);
      else p.nonbatch_reqs.push_back(r);
    }
    if (batchable.empty()) continue;
    chunkify_maximize_chunk_size((uint32_t)batchable.size(), 16, bounds);
    const uint32_t base = (uint32_t)p.chunk_reqs.size();
    p.chunk_reqs.insert(p.chunk_reqs.end(), batchable.begin(), batchable.end());
    for (size_t k = 1; k < bounds.size(); ++k) p.chunk_off.push_back(base + bounds[k]);
  }
}

// Host-side shape checks of one caller batch (0, or -2 with ctx->err).  The kernels and
// the verify_many join index sets and key lists through these offsets, so they must
// start at 0, be monotone and end at the array sizes.
static int check_batch(bls_gpu_ctx* ctx, const bls_batch* in, const char* what) {
  const uint32_t n = in->n_sets, R = in->n_reqs;
  if (R == 0) return 0;
  if (!in->req_set_offsets) {
    snprintf(ctx->err, sizeof(ctx->err), "%s: req_set_offsets missing", what);
    return -2;
  }
  if (in->req_set_offsets[0] != 0 || in->req_set_offsets[R] != n) {
    snprintf(ctx->err, sizeof(ctx->err), "%s: req_set_offsets must run from 0 to n_sets", what);
    return -2;
  }
  if (in->set_pk_offsets == nullptr && in->pubkeys == nullptr && n > 0) {
    snprintf(ctx->err, sizeof(ctx->err), "%s: no pubkeys given", what);
    return -2;
  }
  if (n > 0 && (!in->messages || !in->signatures)) {
    snprintf(ctx->err, sizeof(ctx->err), "%s: messages / signatures missing", what);
    return -2;
  }
  for (uint32_t r = 0; r < R; ++r) {
    if (in->req_set_offsets[r] > in->req_set_offsets[r + 1]) {
      snprintf(ctx->err, sizeof(ctx->err), "%s: req_set_offsets not monotone at %u", what, r);
      return -2;
    }
  }
  if (in->set_pk_offsets) {
    if (in->set_pk_offsets[0] != 0) {
      snprintf(ctx->err, sizeof(ctx->err), "%s: set_pk_offsets[0] != 0", what);
      return -2;
    }
    for (uint32_t i = 0; i < n; ++i) {
      if (in->set_pk_offsets[i] > in->set_pk_offsets[i + 1]) {
        snprintf(ctx->err, sizeof(ctx->err), "%s: set_pk_offsets not monotone at %u", what, i);
        return -2;
      }
    }
    if (in->set_pk_offsets[n] > 0 && !in->pk_indices) {
      snprintf(ctx->err, sizeof(ctx->err), "%s: pk_indices missing", what);
      return -2;
    }
  }
  return 0;
}

struct InFlight {
  uint64_t n;
  explicit InFlight(uint64_t k) : n(k) { g_sets_in_flight.fetch_add(n, std::memory_order_relaxed); }
  ~InFlight() { g_sets_in_flight.fetch_sub(n, std::memory_order_relaxed); }
};

// How the verify path's host thread waits for its stream.  hipStreamSynchronize spins
// (so does hipEventSynchronize on a hipEventBlockingSync event in this runtime): with 16
// contexts each waiting through a ~95 ms pass the process held ~15.7 CPUs and the job's
// 16-CPU quota throttled it (profiles/r06_ab_sync_wait.json) -- CPU a beacon node's main
// thread and its other work need.  A pass of more than 2,048 sets (only the aggregated
// path takes those; tens of ms) polls an event with 50 us sleeps instead; smaller calls
// keep the spin: they can take the per-set path, a few ms, where polling at 1024-set
// calls cost 4 x 1 calls 7.2 -> 7.8 ms.  $BLS_SYNC=spin / poll forces either.
static int sync_mode() {
  static const int m = [] {
    const char* e = getenv("BLS_SYNC");
    return e && !strcmp(e, "spin") ? 1 : e && !strcmp(e, "poll") ? 2 : 0;
  }();
  return m;
}
static bool wait_blocks(uint32_t n_sets) {
  const int m = sync_mode();
  return m == 2 || (m == 0 && n_sets > 2048);
}
static hipError_t pass_wait(bls_gpu_ctx* ctx, hipStream_t s) {
  if (!ctx->wait_block || s != ctx->stream) return hipStreamSynchronize(s);
  hipError_t e = hipEventRecord(ctx->ev_wait, s);
  if (e != hipSuccess) return e;
  const struct timespec nap = {0, 50000};
  while ((e = hipEventQuery(ctx->ev_wait)) == hipErrorNotReady) nanosleep(&nap, nullptr);
  return e;
}

static int verify_body(bls_gpu_ctx* ctx, const bls_batch* in, int32_t* verdicts, bls_stats* stats,
                       uint32_t scalar_base, uint8_t* partial_out, int32_t* partial_status, uint32_t* partial_err,
                       const std::vector<uint32_t>* req_bounds);

// One call under the context's lock.  A call that fails part-way may leave the MSM's
// bucket counters / tickets (reset only by the kernels' last workgroups) mid-pass: they
// are zeroed again before the context takes another call.
static int verify_impl(bls_gpu_ctx* ctx, const bls_batch* in, int32_t* verdicts, bls_stats* stats,
                       uint32_t scalar_base, uint8_t* partial_out, int32_t* partial_status,
                       uint32_t* partial_err = nullptr, const std::vector<uint32_t>* req_bounds = nullptr) {
  CTX_LOCK(ctx);
  ctx->wait_block = wait_blocks(in->n_sets);
  const int rc = verify_body(ctx, in, verdicts, stats, scalar_base, partial_out, partial_status, partial_err,
                             req_bounds);
  if (rc < 0 && ctx->msm_state) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipMemsetAsync(ctx->msm_state, 0, sizeof(uint32_t) * MSM_STATE_WORDS, ctx->stream);
    (void)hipStreamSynchronize(ctx->stream);
  }
  return rc;
}

static int verify_body(bls_gpu_ctx* ctx, const bls_batch* in, int32_t* verdicts, bls_stats* stats,
                       uint32_t scalar_base, uint8_t* partial_out, int32_t* partial_status, uint32_t* partial_err,
                       const std::vector<uint32_t>* req_bounds) {
  const bool partial = partial_out != nullptr;
  HIPC(ctx, hipSetDevice(ctx->device));
  const uint32_t n = in->n_sets, R = in->n_reqs;
  if (stats) memset(stats, 0, sizeof(*stats));
  if (R == 0) return 0;
  if (const int rc = check_batch(ctx, in, "batch")) return rc;
  const InFlight in_flight(n);
  BatchPlan plan;
  if (req_bounds) plan_batch_msgs(in, *req_bounds, plan);
  else plan_batch(in, plan);
  std::vector<uint32_t> msg_uniq, msg_rep;
  const uint32_t n_uniq = (ctx->debug_flags & BLS_DEBUG_NO_MSG_DEDUP) ? n : plan_msg_dedup(in->messages, n, msg_uniq, msg_rep);
  const bool dedup = n_uniq < n;
  // Merged check: with only batchable requests and >= 2 chunks, first test the
  // product of every f_i with ONE final exponentiation (k_fprod tree); it passes iff
  // every chunk would (the same random-scalar batch, just larger), so chunk_ok is
  // all 1 and the per-chunk final exponentiations are skipped.  A failing merged
  // check (or a request with an error status) falls back to k_chunk_coop, so
  // verdicts and stats stay those of the chunked worker (worker.ts:56-88).
  const bool merged_eligible = !partial && plan.chunk_off.size() > 2 && plan.nonbatch_reqs.empty() && n > 0 &&
                               !(ctx->debug_flags & BLS_DEBUG_NO_MERGED_CHECK);
  const bool merged_skipped = merged_eligible && ctx->last_merged_failed && merged_skip_after_fail() &&
                              !(ctx->debug_flags & BLS_DEBUG_MERGED_EVERY_PASS);
  const bool merged = merged_eligible && !merged_skipped;
  const uint32_t n_chunks = (uint32_t)plan.chunk_off.size() - 1;
  const uint32_t n_pk_idx = in->set_pk_offsets ? in->set_pk_offsets[n] : 0;
  // aggregated-signature path: virtual sets n + chunk and n + n_chunks + individual
  // request; the chunk groups' sum plan is staged with the inputs
  const bool sigagg = n > 0 && use_sigagg(ctx, n);
  GsumPlan chunk_gsum, unit_gsum;
  UnitPlan units;
  const bool use_units = sigagg && dedup && !(ctx->debug_flags & BLS_DEBUG_NO_UNITS) &&
                         plan_units(in, plan, msg_rep, n, units);
  const uint32_t n_units = use_units ? units.n_units : 0;
  // f / chain layout: sets [0, n) | chunk signature sums [n, n + C) | units
  // [n + C, n + C + U) | individual requests' signature sums [n + C + U, .. + R)
  const uint32_t unit_base = n + n_chunks, indiv_vbase = n + n_chunks + n_units;
  const uint32_t n_total = sigagg ? indiv_vbase + R : n;
  if (sigagg) {
    std::vector<uint32_t> goff(plan.chunk_off.begin(), plan.chunk_off.end());
    plan_gsum(in, goff, plan.chunk_reqs, chunk_gsum);
  }
  if (use_units) plan_gsum_sets(units.goff, units.members, unit_gsum);
  // Merged signature sum: under the merged check the chunks' signature sums only ever
  // meet in the product of every f, and prod_c e(-g1, S_c) = e(-g1, sum_c S_c) after the
  // final exponentiation, so the first pass sums every chunk's r_i sig_i into ONE point
  // (chunk group 0; the other chunk groups are empty, so k_vset gives them f = 1) and
  // pairs it once.  A failing merged check re-sums per chunk and pairs each sum before
  // the per-chunk final exponentiations (k_chunk_coop), so chunk verdicts are unchanged.
  const bool use_total = sigagg && merged && n_chunks > 1 && sig_total_on();
  // ... and under it the sum is one Pippenger MSM over the live sets (kernels/k_msm.hip)
  // instead of per-set [r] sig chains + k_gsum levels; the per-set RS are made (k_chain
  // role 2 alone) only when the merged check fails and the chunks' own sums are needed
  // (an MSM entry packs its bucket slot in 22 bits and a bucket takes up to 2 entries per
  // set: passes above MSM_MAX_SETS keep the group sums)
  const bool use_msm = use_total && n <= MSM_MAX_SETS &&
                       ((msm_on() && !ctx->last_merged_failed) || (ctx->debug_flags & BLS_DEBUG_MSM));
  GsumPlan total_gsum;
  if (use_total) {
    std::vector<uint32_t> goff(n_chunks + 1, (uint32_t)chunk_gsum.gsets.size());
    goff[0] = 0;
    plan_gsum_sets(goff, chunk_gsum.gsets, total_gsum);
  }
  const size_t gseg_cap = 2ull * (n / 2 + 12ull * R + 8);  // uint32s: every level of any plan (fan-in >= 4)
  const size_t gtmp_cap = n / GSUM_FAN + R + 1;                  // level-0 segments of any plan
  if (sigagg && chunk_gsum.seg.size() > gseg_cap) {
    snprintf(ctx->err, sizeof(ctx->err), "group-sum plan exceeds its workspace");
    return -3;
  }

  // product domain of every first-pass Miller-loop item (sets, chunk signature sums,
  // units): k_mln shares one loop among four consecutive live items of one domain
  const bool ml_shared = sigagg && ml_shared_on();
  std::vector<uint32_t> ml_dom;
  if (ml_shared) {
    ml_dom.assign(indiv_vbase, 0xFFFFFFFFu);
    for (uint32_t ch = 0; ch < n_chunks; ++ch) {
      for (uint32_t k = plan.chunk_off[ch]; k < plan.chunk_off[ch + 1]; ++k) {
        const uint32_t r = plan.chunk_reqs[k];
        for (uint32_t i = in->req_set_offsets[r]; i < in->req_set_offsets[r + 1]; ++i) ml_dom[i] = ch;
      }
      ml_dom[n + ch] = ch;
      if (use_units)
        for (uint32_t u = units.unit_off[ch]; u < units.unit_off[ch + 1]; ++u) ml_dom[unit_base + u] = ch;
    }
    for (uint32_t r : plan.nonbatch_reqs)
      for (uint32_t i = in->req_set_offsets[r]; i < in->req_set_offsets[r + 1]; ++i) ml_dom[i] = 0x80000000u | r;
  }

  // aggregate sets big enough for a wavefront each (k_pk_agg)
  std::vector<uint32_t> agg_list;
  if (in->set_pk_offsets)
    for (uint32_t i = 0; i < n; ++i)
      if (in->set_pk_offsets[i + 1] - in->set_pk_offsets[i] >= BLS_AGG_WAVE_MIN) agg_list.push_back(i);

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
  Fp12* ptree[2] = {nullptr, nullptr};  // product-tree levels (partial mode, merged check)
  int32_t* merged_ok = nullptr;          // FE(prod f_i) == 1 of the merged check
  uint32_t* gsets_dev = nullptr;         // group-sum plans (aggregated-signature path)
  uint32_t* gseg_dev = nullptr;
  uint32_t* tseg_dev = nullptr;          // the merged signature sum's plan
  G2J* gtmp[2] = {nullptr, nullptr};
  uint32_t *unit_rep_dev = nullptr, *ugsets_dev = nullptr, *useg_dev = nullptr;  // Miller-loop units
  uint32_t* own_sets_dev = nullptr;      // the individually verified sets' own Miller loops + the requests' sums (one launch)
  // SIMT final exponentiations (kernels/k_fin_simt.hip) for a failing pass's many chunk
  // checks / requests verified alone: 4 Fp12 per task, carved when a pass could need them
  const uint32_t fe_min = fe_simt_min();
  const bool fe_simt_possible = fe_min > 0 && (n_chunks >= fe_min || R >= fe_min);
  Fp12* fe_save = nullptr;
  MsmBufs msm;
  memset(&msm, 0, sizeof(msm));
  G1J* utmp[2] = {nullptr, nullptr};
  // group tests over failed chunks (passes reuse the buffers): pass A <= 1 + 13 tests per
  // chunk (chunks of < 8192 requests) of <= 8 m members in all, pass B 2 tests, pass C one
  // test per request
  // (carved only when some chunk is large enough to be group-tested, group_test_min)
  bool gt_possible = false;
  {
    const uint32_t gmin = group_test_min(ctx);
    for (uint32_t ch = 0; ch < n_chunks && !gt_possible; ++ch)
      gt_possible = plan.chunk_off[ch + 1] - plan.chunk_off[ch] >= gmin;
  }
  const size_t grp_cap = gt_possible ? (size_t)R + 14ull * n_chunks + 2 : 0,
               grp_mem_cap = gt_possible ? 8ull * R + 16 : 0;
  GroupBufs gbufs;
  memset(&gbufs, 0, sizeof(gbufs));
  auto carve = [&](Carver& c, PipeBufs& b, size_t& input_end) {
    b.req_off = c.take<uint32_t>(R + 1);
    b.chunk_off = c.take<uint32_t>(n_chunks + 1);
    b.chunk_reqs = c.take<uint32_t>(plan.chunk_reqs.size());
    b.seed = c.take<uint32_t>(8);
    b.pubkeys = in->set_pk_offsets ? nullptr : c.take<uint8_t>(96ull * n);
    b.set_pk_off = in->set_pk_offsets ? c.take<uint32_t>(n + 1) : nullptr;
    b.pk_idx = in->set_pk_offsets ? c.take<uint32_t>(n_pk_idx) : nullptr;
    b.agg_sets = agg_list.empty() ? nullptr : c.take<uint32_t>(agg_list.size());
    b.msgs = c.take<uint8_t>(32ull * n);
    b.msg_uniq = dedup ? c.take<uint32_t>(n_uniq) : nullptr;
    b.msg_rep = dedup ? c.take<uint32_t>(n) : nullptr;
    b.sigs = c.take<uint8_t>(96ull * n);
    b.sig_lens = in->signature_lens ? c.take<uint32_t>(n) : nullptr;
    b.indiv_reqs = c.take<uint32_t>(R);
    gbufs.off = c.take<uint32_t>(gt_possible ? grp_cap + 1 : 0);
    gbufs.members = c.take<uint32_t>(grp_mem_cap);
    gbufs.ref = c.take<uint32_t>(gt_possible ? grp_cap : 0);
    own_sets_dev = sigagg ? c.take<uint32_t>((size_t)n + R) : nullptr;
    b.fold_groups = c.take<uint32_t>(2ull * (n / BLS_FOLD1 + R + 1) + 2ull * (n / BLS_FOLD + R + 1));
    b.ml_dom = ml_shared ? c.take<uint32_t>(indiv_vbase) : nullptr;
    gsets_dev = sigagg ? c.take<uint32_t>(n) : nullptr;
    gseg_dev = sigagg ? c.take<uint32_t>(gseg_cap) : nullptr;
    tseg_dev = use_total ? c.take<uint32_t>(total_gsum.seg.size()) : nullptr;
    if (use_units) {
      b.set_unit = c.take<uint32_t>(n);
      unit_rep_dev = c.take<uint32_t>(n_units);
      b.unit_off = c.take<uint32_t>(n_chunks + 1);
      ugsets_dev = c.take<uint32_t>(units.members.size());
      useg_dev = c.take<uint32_t>(unit_gsum.seg.size());
    }
    input_end = c.off;
    b.sig = c.take<G2A>(n);
    b.sig_status = c.take<int32_t>(n);
    b.pk = c.take<G1J>(n);
    b.pk_status = c.take<int32_t>(n);
    b.pk_inf = partial ? c.take<uint8_t>(n) : nullptr;
    b.q = c.take<Fp>(8ull * n);
    b.chain = sigagg ? c.take<Fp>((size_t)CHAIN_WORDS * n_total) : nullptr;
    b.chain_live = sigagg ? c.take<uint32_t>(n_total) : nullptr;
    b.chain_st = sigagg ? c.take<uint8_t>(4ull * n) : nullptr;
    b.rtab2 = sigagg ? c.take<G2J>(15ull * n) : nullptr;
    b.rtab1 = c.take<G1J>((sigagg ? 15ull : 30ull) * n);
    b.rpts = sigagg ? nullptr : c.take<G1J>(2ull * n);
    gtmp[0] = sigagg ? c.take<G2J>(gtmp_cap) : nullptr;
    gtmp[1] = sigagg ? c.take<G2J>(gtmp_cap) : nullptr;
    utmp[0] = use_units ? c.take<G1J>(unit_gsum.level_off[1] + 1) : nullptr;
    utmp[1] = use_units ? c.take<G1J>(unit_gsum.level_off[1] + 1) : nullptr;
    b.set_flag = c.take<uint32_t>(n);
    b.flag_count = c.take<uint32_t>(1);
    b.f = c.take<Fp12>(n_total);
    b.ml_lines = sigagg ? c.take<uint32_t>(mlq_line_words(n_total)) : nullptr;
    if (use_msm) {
      msm.off = c.take<uint32_t>(MSM_BUCKETS + 1);
      msm.seg_off = c.take<uint32_t>(MSM_BUCKETS + 1);
      msm.ent = c.take<uint32_t>(8ull * n);
      msm.sorted = c.take<uint32_t>(8ull * n);
      msm.seg_sum = c.take<G2J>(msm_seg_cap(n));
      msm.bucket = c.take<G2J>(MSM_BUCKETS);
      msm.win = c.take<G2J>(4);
    }
    b.req_status = c.take<int32_t>(R);
    gbufs.f = gt_possible ? c.take<Fp12>(R) : nullptr;
    gbufs.fe = gt_possible ? c.take<Fp12>(grp_cap) : nullptr;
    b.chunk_fe = gt_possible ? c.take<Fp12>(n_chunks) : nullptr;
    fe_save = fe_simt_possible ? c.take<Fp12>(4ull * (n_chunks > R ? n_chunks : R)) : nullptr;
    if (partial || merged) {
      ptree[0] = c.take<Fp12>((n_total + FPROD_FAN - 1) / FPROD_FAN);
      ptree[1] = c.take<Fp12>((n_total + FPROD_FAN - 1) / FPROD_FAN);
    }
  };
  // results: written by the kernels straight into host-mapped memory
  auto carve_res = [&](Carver& c, PipeBufs& b) {
    b.chunk_ok = c.take<int32_t>(n_chunks);
    b.indiv_verdict = c.take<int32_t>(R);
    gbufs.verdict = c.take<int32_t>(grp_cap);
    b.req_status_host = c.take<int32_t>(R);
    b.flag_count_host = c.take<uint32_t>(1);
    merged_ok = merged ? c.take<int32_t>(1) : nullptr;
  };
  PipeBufs b;
  memset(&b, 0, sizeof(b));
  size_t input_end = 0;
  {
    Carver c{nullptr, 0}, cr{nullptr, 0};
    carve(c, b, input_end);
    carve_res(cr, b);
    if (ensure_dev(ctx, c.off) || ensure_host(ctx, input_end) ||
        ensure_mapped(ctx, cr.off, &ctx->host_res, &ctx->host_res_dev, &ctx->host_res_cap))
      return -1;
  }
  // inputs [0, input_end) live in the mapped staging area, the rest in device memory
  Carver c{ctx->dev_ws, 0, ctx->host_stage_dev, input_end};
  carve(c, b, input_end);
  Carver cr{ctx->host_res_dev, 0};
  carve_res(cr, b);
  b.first_bad_pk = b.pubkeys ? ctx->first_bad + ctx->first_bad_slot : nullptr;
  b.first_bad_pk_next = ctx->first_bad + (ctx->first_bad_slot ^ 1u);
  b.init_set_flag = (ctx->debug_flags & BLS_DEBUG_FORCE_EXACT) ? 1u : 0u;
  b.n_sets = n;
  b.n_reqs = R;
  b.n_chunks = n_chunks;
  b.pk_table = ctx->table;
  b.pk_table_n = ctx->table_n;
  b.scalar_base = scalar_base;
  b.pack = (ctx->debug_flags & BLS_DEBUG_PACK_MASK) >> 8;
  b.mlf_pl = (ctx->debug_flags & BLS_DEBUG_MLF_PL_MASK) >> 12;
  b.multi_set_rules = partial ? 1u : 0u;
  b.sigagg = sigagg ? 1u : 0u;
  b.unit_base = unit_base;
  b.n_units = n_units;
  b.indiv_vbase = indiv_vbase;
  if (use_units) {
    stage_copy(ctx, b.set_unit, units.set_unit.data(), sizeof(uint32_t) * n);
    stage_copy(ctx, unit_rep_dev, units.unit_rep.data(), sizeof(uint32_t) * n_units);
    stage_copy(ctx, b.unit_off, units.unit_off.data(), sizeof(uint32_t) * (n_chunks + 1));
    stage_copy(ctx, ugsets_dev, units.members.data(), sizeof(uint32_t) * units.members.size());
    stage_copy(ctx, useg_dev, unit_gsum.seg.data(), sizeof(uint32_t) * unit_gsum.seg.size());
  }
  if (ml_shared) stage_copy(ctx, b.ml_dom, ml_dom.data(), sizeof(uint32_t) * ml_dom.size());
  if (sigagg) {
    stage_copy(ctx, gsets_dev, chunk_gsum.gsets.data(), sizeof(uint32_t) * chunk_gsum.gsets.size());
    stage_copy(ctx, gseg_dev, chunk_gsum.seg.data(), sizeof(uint32_t) * chunk_gsum.seg.size());
    if (use_total) stage_copy(ctx, tseg_dev, total_gsum.seg.data(), sizeof(uint32_t) * total_gsum.seg.size());
  }

  stage_copy(ctx, b.req_off, in->req_set_offsets, sizeof(uint32_t) * (R + 1));
  stage_copy(ctx, b.chunk_off, plan.chunk_off.data(), sizeof(uint32_t) * (n_chunks + 1));
  stage_copy(ctx, b.chunk_reqs, plan.chunk_reqs.data(), sizeof(uint32_t) * plan.chunk_reqs.size());
  stage_copy(ctx, b.seed, seed_words, sizeof(seed_words));
  if (b.pubkeys) stage_copy(ctx, b.pubkeys, in->pubkeys, 96ull * n);
  if (b.set_pk_off) {
    stage_copy(ctx, b.set_pk_off, in->set_pk_offsets, sizeof(uint32_t) * (n + 1));
    stage_copy(ctx, b.pk_idx, in->pk_indices, sizeof(uint32_t) * n_pk_idx);
  }
  b.n_agg = (uint32_t)agg_list.size();
  b.agg_min = agg_list.empty() ? 0u : BLS_AGG_WAVE_MIN;
  if (!agg_list.empty()) stage_copy(ctx, b.agg_sets, agg_list.data(), sizeof(uint32_t) * agg_list.size());
  stage_copy(ctx, b.msgs, in->messages, 32ull * n);
  b.n_uniq = dedup ? n_uniq : 0;
  if (dedup) {
    stage_copy(ctx, b.msg_uniq, msg_uniq.data(), sizeof(uint32_t) * n_uniq);
    stage_copy(ctx, b.msg_rep, msg_rep.data(), sizeof(uint32_t) * n);
  }
  if (in->signature_lens) {
    // bytes past a short signature's length are never read (the set fails INVALID_SIZE)
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t len = in->signature_lens[i] < 96 ? in->signature_lens[i] : 96;
      uint8_t* dst = ctx->host_stage + ((const uint8_t*)b.sigs - ctx->host_stage_dev) + 96ull * i;
      memset(dst, 0, 96);
      memcpy(dst, in->signatures + 96ull * i, len);
    }
    stage_copy(ctx, b.sig_lens, in->signature_lens, sizeof(uint32_t) * n);
  } else {
    stage_copy(ctx, b.sigs, in->signatures, 96ull * n);
  }

  hipStream_t s = ctx->stream;
  HIPC(ctx, hipEventRecord(ctx->ev0, s));
  HIPC(ctx, hipEventRecord(ctx->ev[0], s));  // no H2D stage: the kernels read the mapped inputs
  if (n > 0) {
    HIPC(ctx, launch_k_pk(b, s));  // also resets set_flag, flag_count, the next first_bad_pk slot
    HIPC(ctx, launch_k_pk_agg(b, s)); dbg_sync(s, "k_pk");
    ctx->first_bad_slot ^= 1u;
    HIPC(ctx, hipEventRecord(ctx->ev[1], s));
    HIPC(ctx, launch_k_pre(b, s)); dbg_sync(s, "k_pre");
    HIPC(ctx, hipEventRecord(ctx->ev[2], s));
    if (sigagg) {
      // per-set chains, the chunks' sums of r sig -> virtual sets n + c, then every
      // Miller loop (sets and virtual sets) in one launch
      HIPC(ctx, launch_k_chain(b, s, use_msm ? 0xBu : 0xFu)); dbg_sync(s, "k_chain");
      HIPC(ctx, hipEventRecord(ctx->ev[3], s));
      if (use_msm) {
        msm.cnt = ctx->msm_state;
        msm.ticket = ctx->msm_state + MSM_BUCKETS;
        HIPC(ctx, launch_k_msm(b, msm, n_chunks, n, s)); dbg_sync(s, "k_msm");
      } else if (launch_gsum(ctx, b, use_total ? total_gsum : chunk_gsum, use_total ? tseg_dev : gseg_dev, gsets_dev,
                             gtmp, n, s)) {
        return -1;
      }
      if (use_units) {
        // sum r_i pk_i per unit (levels over the members), then the units' chain entries
        b.gsets = ugsets_dev;
        const G1J* uin = nullptr;
        const size_t levels = unit_gsum.level_off.size() - 1;
        for (size_t L = 0; L < levels; ++L) {
          const uint32_t beg = unit_gsum.level_off[L], n_seg = unit_gsum.level_off[L + 1] - beg;
          HIPC(ctx, launch_k_gsum1(b, useg_dev + 2 * beg, n_seg, uin, utmp[L & 1], s)); dbg_sync(s, "k_gsum1");
          uin = utmp[L & 1];
        }
        HIPC(ctx, launch_k_uset(b, uin, unit_rep_dev, s)); dbg_sync(s, "k_uset");
        b.gsets = gsets_dev;
      }
      HIPC(ctx, hipEventRecord(ctx->ev[4], s));
      // the f-side shape is chosen once per call (other contexts change the sets in flight
      // meanwhile): the first pass's Miller-loop launch and stats->pass_shape use it
      if (!b.mlf_pl && k_mln_list_ok(b)) b.mlf_pl = mlf_per_lane();
      HIPC(ctx, launch_k_mln(b, ctx->coop, 0, indiv_vbase, s)); dbg_sync(s, "k_mln");
    } else {
      HIPC(ctx, launch_k_pset(b, ctx->coop, s)); dbg_sync(s, "k_pset");
      HIPC(ctx, hipEventRecord(ctx->ev[3], s));
      HIPC(ctx, hipEventRecord(ctx->ev[4], s));
    }
    // stage_ms[3] k_chain (or k_pset), [4] the signature sums (k_gsum / k_msm, units),
    // [5] the Miller loops (k_mlq + k_mlf): the per-kernel launch times bench.py prices
    HIPC(ctx, hipEventRecord(ctx->ev[5], s));
  } else {
    for (int i = 1; i <= 5; ++i) HIPC(ctx, hipEventRecord(ctx->ev[i], s));
  }
  HIPC(ctx, launch_k_status(b, s)); dbg_sync(s, "k_status");
  // Merged check: FE(prod of every f_i) == 1 with one final exponentiation (k_fprod
  // tree 1024 -> 16 -> 1), before any per-chunk one.
  const uint32_t n_prod = sigagg ? indiv_vbase : n;  // the f's of every set, chunk group and unit
  auto launch_merged = [&]() -> int {
    const Fp12* cur = b.f;
    uint32_t m = n_prod, lvl = 0;
    while (m > FPROD_FAN) {
      HIPC(ctx, launch_k_fprod(cur, m, ptree[lvl & 1], nullptr, ctx->coop, s)); dbg_sync(s, "k_fprod");
      cur = ptree[lvl & 1];
      m = (m + FPROD_FAN - 1) / FPROD_FAN;
      ++lvl;
    }
    HIPC(ctx, launch_k_fprod(cur, m, nullptr, merged_ok, ctx->coop, s)); dbg_sync(s, "k_fprod merged");
    return 0;
  };
  if (merged && launch_merged()) return -1;
  HIPC(ctx, hipEventRecord(ctx->ev[6], s));

  // the per-set RS = [r] sig (chain CH_RS) the fallback sums need: made by the first pass
  // unless the MSM replaced role 2 there
  bool rs_done = !use_msm;
  auto ensure_rs = [&]() -> int {
    if (!rs_done) {
      HIPC(ctx, launch_k_chain(b, s, 0x4u)); dbg_sync(s, "k_chain rs");
      rs_done = true;
    }
    return 0;
  };
  // the Miller-loop launches after the first pass take their own items-per-lane
  // (mlf_per_lane_alone: their items never share f) unless a test forces one
  const uint32_t pass_pl = b.mlf_pl;
  const bool pl_forced = (ctx->debug_flags & BLS_DEBUG_MLF_PL_MASK) != 0;
  auto alone_pl = [&](uint32_t count) {
    const uint32_t pl = mlf_per_lane_alone(count);
    if (pl && !pl_forced && k_mln_list_ok(b)) b.mlf_pl = pl;
  };
  // ... and up to coop_ml_max() items they are cooperative single-pair loops, one
  // wavefront per item (launch_k_mln_coop), else the SIMT pair at that shape
  auto launch_ml_alone = [&](uint32_t first, uint32_t count, const uint32_t* items) -> hipError_t {
    if (count == 0) return hipSuccess;
    if (!pl_forced && k_mln_list_ok(b)) {
      const hipError_t e = launch_k_mln_coop(b, ctx->coop, first, count, items, s);
      if (e != hipErrorNotSupported) return e;
    }
    alone_pl(count);
    return items ? launch_k_mln_list(b, items, count, s) : launch_k_mln(b, ctx->coop, first, count, s);
  };
  std::vector<int32_t> chunk_ok(n_chunks + 1, 0);
  std::vector<int32_t> merged_status(merged ? R : 0, 0);
  int32_t merged_verdict = 0;
  uint32_t flagged = 0;
  // after a stream sync: the merged verdict and the statuses, from the mapped result area
  auto read_merged = [&]() {
    merged_verdict = *res_host(ctx, merged_ok);
    memcpy(merged_status.data(), res_host(ctx, b.req_status_host), sizeof(int32_t) * R);
  };
  HIPC(ctx, pass_wait(ctx, s));
  if (merged) read_merged();
  if (n > 0) flagged = *res_host(ctx, b.flag_count_host);
  if (flagged) {
    // rare: sets the cooperative kernel could not finish (exceptional additions,
    // infinity signatures, special SSWU inputs) -> exact path, then the status (the
    // exact path may find a signature outside G2) and the merged check again
    HIPC(ctx, launch_k_exact(b, s)); dbg_sync(s, "k_exact");
    HIPC(ctx, launch_k_status(b, s)); dbg_sync(s, "k_status");
    if (merged && launch_merged()) return -1;
    HIPC(ctx, pass_wait(ctx, s));
    if (merged) read_merged();
  }
  bool merged_pass = merged && merged_verdict == 1;
  bool chunk_fe_kept = false;
  for (uint32_t r = 0; merged_pass && r < R; ++r) merged_pass = merged_status[r] == BLS_OK;
  if (merged) ctx->last_merged_failed = !merged_pass;
  if (merged_pass) {
    for (uint32_t ch = 0; ch < n_chunks; ++ch) chunk_ok[ch] = 1;
  } else if (n_chunks > 0 && !partial) {
    // some set is invalid or erroneous (or no merged check): the per-chunk verdicts decide
    if (ensure_rs()) return -1;
    if (use_total) {
      // the chunks' own signature sums and their Miller loops (virtual sets n + c)
      if (launch_gsum(ctx, b, chunk_gsum, gseg_dev, gsets_dev, gtmp, n, s)) return -1;
      HIPC(ctx, launch_ml_alone(n, n_chunks, nullptr)); dbg_sync(s, "k_mln chunk sums");
    }
    // many chunk checks: one lane each (a failing pass at the plateau has hundreds, and a
    // cooperative task holds a SIMD for a whole final exponentiation); few: one wavefront
    // each, the shorter latency
    if (fe_save && n_chunks >= fe_min) HIPC(ctx, launch_k_chunk_simt(b, fe_save, s));
    else {
      HIPC(ctx, launch_k_chunk_coop(b, ctx->coop, s));
      chunk_fe_kept = b.chunk_fe != nullptr;  // the checked chunks' final exponentiations
    }
    dbg_sync(s, "k_chunk");
    HIPC(ctx, pass_wait(ctx, s));
    memcpy(chunk_ok.data(), res_host(ctx, b.chunk_ok), sizeof(int32_t) * n_chunks);
  }
  if (merged_skipped) {
    // the context keeps skipping the merged check while its passes keep failing a chunk
    bool all_ok = true;
    for (uint32_t ch = 0; ch < n_chunks; ++ch) all_ok = all_ok && chunk_ok[ch] == 1;
    ctx->last_merged_failed = !all_ok;
  }
  if (stats) {
    stats->merged_check = merged ? (merged_pass ? 1 : 2) : (merged_skipped ? 3 : 0);
    stats->pass_shape =
        sigagg ? ((use_msm ? 1u : 0u) | (k_mln_list_ok(b) ? pass_pl << 8 : 0u)) : 0u;
  }
  if (stats) {
    stats->n_flagged = flagged;
    stats->n_unique_msgs = n_uniq;
    stats->n_ml_units = n_units;
  }
  if (partial) {
    // the call rejects with the code of its first error, classes in the reference's
    // order: a pubkey that does not decode / aggregate (deserializeSet and
    // getAggregatedPubkey run before anything else, worker.ts:45, index.ts:160), then a
    // signature that does not decode (maybeBatch.ts:19-24 maps fromBytes over the
    // sets), then an infinity pubkey (verifyMultipleSignatures).  The shard reports its
    // first error of the lowest class with its set index, so the ranks can reduce
    // (class, call index) in that order (lodestar_amd/shard.py).
    std::vector<int32_t> st(res_host(ctx, b.req_status_host), res_host(ctx, b.req_status_host) + R);
    *partial_status = 0;
    for (uint32_t r = 0; r < R && !*partial_status; ++r)
      if (st[r] != 0) *partial_status = -st[r];
    if (*partial_status && n > 0) {
      std::vector<int32_t> pks(n), sgs(n);
      std::vector<uint8_t> inf(n);
      HIPC(ctx, hipMemcpyAsync(pks.data(), b.pk_status, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
      HIPC(ctx, hipMemcpyAsync(sgs.data(), b.sig_status, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
      HIPC(ctx, hipMemcpyAsync(inf.data(), b.pk_inf, n, hipMemcpyDeviceToHost, s));
      HIPC(ctx, pass_wait(ctx, s));
      uint32_t cls = 3, idx = 0;
      int32_t code = 0;
      for (uint32_t i = 0; i < n && cls > 0; ++i)
        if (pks[i] != BLS_OK) { cls = 0; idx = i; code = pks[i]; }
      for (uint32_t i = 0; i < n && cls > 1; ++i)
        if (sgs[i] != BLS_OK) { cls = 1; idx = i; code = sgs[i]; }
      for (uint32_t i = 0; i < n && cls > 2; ++i)
        if (inf[i]) { cls = 2; idx = i; code = BLS_PK_IS_INFINITY; }
      if (cls < 3) *partial_status = -code;  // else: an empty-request code (kept)
      if (partial_err) {
        partial_err[0] = cls;
        partial_err[1] = idx;
      }
    }
    if (*partial_status || n == 0) return 0;
    const Fp12* cur = b.f;
    uint32_t m = n_prod, lvl = 0;
    while (m > 1) {
      HIPC(ctx, launch_k_fprod(cur, m, ptree[lvl & 1], nullptr, ctx->coop, s)); dbg_sync(s, "k_fprod");
      cur = ptree[lvl & 1];
      m = (m + FPROD_FAN - 1) / FPROD_FAN;
      ++lvl;
    }
    HIPC(ctx, hipMemcpyAsync(partial_out, cur, sizeof(Fp12), hipMemcpyDeviceToHost, s));
    HIPC(ctx, pass_wait(ctx, s));
    if (stats) {
      float ms = 0.f;
      HIPC(ctx, hipEventRecord(ctx->ev1, s));
      HIPC(ctx, hipEventSynchronize(ctx->ev1));
      (void)hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
      stats->device_ms = ms;
    }
    return 0;
  }

  // Requests verified on their own: the non-batchable ones, then the failed chunks'
  // (worker.ts:91-98).  A failed chunk of >= GT_MIN_REQS requests is group-tested
  // instead of paying one final exponentiation per request (verify_groups below); its
  // requests follow the directly verified ones in the list.
  std::vector<uint32_t> indiv = plan.nonbatch_reqs;
  std::vector<GtChunk> gt_chunks;  // [beg, end) of a group-tested chunk in indiv, its chunk
  const uint32_t gt_min = group_test_min(ctx);
  for (int pass = 0; pass < 2; ++pass)
    for (uint32_t ch = 0; ch < n_chunks; ++ch) {
      if (chunk_ok[ch] == 1) continue;
      const uint32_t m = plan.chunk_off[ch + 1] - plan.chunk_off[ch];
      if ((m >= gt_min) != (pass == 1)) continue;
      const uint32_t beg = (uint32_t)indiv.size();
      for (uint32_t k = plan.chunk_off[ch]; k < plan.chunk_off[ch + 1]; ++k) indiv.push_back(plan.chunk_reqs[k]);
      if (pass == 1) gt_chunks.push_back({beg, (uint32_t)indiv.size(), ch});
    }
  const uint32_t n_direct = gt_chunks.empty() ? (uint32_t)indiv.size() : gt_chunks.front().beg;
  // Group sums: on the aggregated path, with many requests group-tested, a group-tested
  // request pairs no signature sum of its own; each group test pairs ONE sum over its
  // requests' sets (run_group_tests) -- 4-6 Miller loops per failed chunk of 16 instead of
  // 16 (group_sums_on).
  const bool gsums = sigagg && !gt_chunks.empty() && group_sums_on(indiv.size() - n_direct);
  const uint32_t n_sum = gsums ? n_direct : (uint32_t)indiv.size();  // requests pairing their own sum
  std::vector<int32_t> indiv_verdict(indiv.size() + 1, 0);
  std::vector<uint32_t> groups;  // k_fold groups; outlives the async copy (synchronised below)
  GsumPlan indiv_gsum;           // likewise
  if (!indiv.empty()) {
    b.n_indiv = (uint32_t)indiv.size();
    stage_copy(ctx, b.indiv_reqs, indiv.data(), sizeof(uint32_t) * indiv.size());  // the stream is idle
    HIPC(ctx, hipEventRecord(ctx->ev[7], s));
    if (sigagg) {
      // each individually verified request pairs the sum of its own r sig:
      // virtual sets indiv_vbase + t; a request whose sets were paired in their
      // chunk's units or shared loops (its chunk failed) now runs their own Miller loops
      std::vector<uint32_t> own;
      const bool own_list = (use_units || ml_shared) && k_mln_list_ok(b);
      // a set needs its own Miller loop again only when the first pass did not leave it
      // one: it was paired in its chunk's unit (f_i = 1), or its f was shared with the
      // next items of its lane (more than one item per k_mlf lane); at one item per lane
      // or per lane pair f_i = e(r_i pk_i, H(m_i)) already
      const bool f_shared = ml_shared && !(pass_pl == 1u || pass_pl == MLF_PAIR);
      if (own_list) {
        // every such set of the failed chunks' requests, in ONE launch with the requests'
        // signature sums below (one Miller-loop latency instead of two on the failing
        // call's path, profiles/r05_cfg5_fallback.json)
        for (size_t t = plan.nonbatch_reqs.size(); t < indiv.size(); ++t)
          for (uint32_t i = in->req_set_offsets[indiv[t]]; i < in->req_set_offsets[indiv[t] + 1]; ++i)
            if (f_shared || (use_units && units.set_unit[i] != UNIT_NONE)) own.push_back(i);
      } else if (use_units || ml_shared) {
        // one launch per run of consecutive sets (a failed chunk's requests are adjacent)
        uint32_t run_beg = 0, run_end = 0;
        for (size_t t = plan.nonbatch_reqs.size(); t <= indiv.size(); ++t) {
          const bool last = t == indiv.size();
          const uint32_t beg = last ? 0 : in->req_set_offsets[indiv[t]], end = last ? 0 : in->req_set_offsets[indiv[t] + 1];
          if (!last && run_end > run_beg && beg == run_end) {
            run_end = end;
            continue;
          }
          if (run_end > run_beg) {
            alone_pl(run_end - run_beg);
            HIPC(ctx, launch_k_mln(b, ctx->coop, run_beg, run_end - run_beg, s, true));
            dbg_sync(s, "k_mln own");
          }
          run_beg = beg;
          run_end = end;
        }
      }
      std::vector<uint32_t> goff(n_sum + 1);
      for (size_t t = 0; t <= n_sum; ++t) goff[t] = (uint32_t)t;
      plan_gsum(in, goff, std::vector<uint32_t>(indiv.begin(), indiv.begin() + n_sum), indiv_gsum);
      if (ensure_rs()) return -1;
      if (indiv_gsum.seg.size() > gseg_cap) {
        snprintf(ctx->err, sizeof(ctx->err), "group-sum plan exceeds its workspace");
        return -3;
      }
      if (n_sum > 0) {  // (under group sums every request may be group-tested)
        stage_copy(ctx, gsets_dev, indiv_gsum.gsets.data(), sizeof(uint32_t) * indiv_gsum.gsets.size());
        stage_copy(ctx, gseg_dev, indiv_gsum.seg.data(), sizeof(uint32_t) * indiv_gsum.seg.size());
        if (launch_gsum(ctx, b, indiv_gsum, gseg_dev, gsets_dev, gtmp, indiv_vbase, s)) return -1;
      }
      if (own_list) {
        for (size_t t = 0; t < n_sum; ++t) own.push_back(indiv_vbase + (uint32_t)t);
        if (!own.empty()) {
          stage_copy(ctx, own_sets_dev, own.data(), sizeof(uint32_t) * own.size());
          HIPC(ctx, launch_ml_alone(0, (uint32_t)own.size(), own_sets_dev));
          dbg_sync(s, "k_mln own + indiv (list)");
        }
      } else {
        HIPC(ctx, launch_ml_alone(indiv_vbase, n_sum, nullptr)); dbg_sync(s, "k_mln indiv");
      }
    }
    // groups of BLS_FOLD consecutive sets per request, multiplied in parallel first: as
    // groups of BLS_FOLD1, then those partial products BLS_FOLD / BLS_FOLD1 at a time
    bool any_fold = false;
    for (uint32_t r : indiv) {
      const uint32_t beg = in->req_set_offsets[r], end = in->req_set_offsets[r + 1];
      for (uint32_t g = beg; g < end; g += BLS_FOLD1) {
        const uint32_t ge = g + BLS_FOLD1 < end ? g + BLS_FOLD1 : end;
        groups.push_back(g);
        groups.push_back(ge);
        any_fold = any_fold || ge - g > 1;
      }
    }
    const uint32_t n_fold1 = (uint32_t)(groups.size() / 2);
    for (uint32_t r : indiv) {
      const uint32_t beg = in->req_set_offsets[r], end = in->req_set_offsets[r + 1];
      for (uint32_t g = beg; g < end; g += BLS_FOLD) {
        const uint32_t ge = g + BLS_FOLD < end ? g + BLS_FOLD : end;
        if (ge - g <= BLS_FOLD1) continue;  // one first-level group: already folded
        groups.push_back(g);
        groups.push_back(ge);
      }
    }
    b.fold = 1;
    b.n_fold = 0;
    if (any_fold) {
      b.fold = BLS_FOLD;
      b.n_fold = (uint32_t)(groups.size() / 2);
      stage_copy(ctx, b.fold_groups, groups.data(), sizeof(uint32_t) * groups.size());
      HIPC(ctx, launch_k_fold(b, ctx->coop, b.fold_groups, n_fold1, 1, s)); dbg_sync(s, "k_fold");
      HIPC(ctx, launch_k_fold(b, ctx->coop, b.fold_groups + 2ull * n_fold1, b.n_fold - n_fold1, BLS_FOLD1, s));
      dbg_sync(s, "k_fold2");
    }
    gbufs.n_direct = n_direct;
    gbufs.sum_f = gsums ? b.f + indiv_vbase + n_direct : nullptr;
    if (fe_save && b.n_indiv >= fe_min) HIPC(ctx, launch_k_indiv_simt(b, gbufs, fe_save, s));
    else HIPC(ctx, launch_k_indiv_coop(b, ctx->coop, gbufs, s));
    dbg_sync(s, "k_indiv");
    if (gt_chunks.empty()) HIPC(ctx, hipEventRecord(ctx->ev[8], s));
  }
  if (gt_chunks.empty()) HIPC(ctx, hipEventRecord(ctx->ev1, s));
  HIPC(ctx, pass_wait(ctx, s));
  if (!indiv.empty()) memcpy(indiv_verdict.data(), res_host(ctx, b.indiv_verdict), sizeof(int32_t) * indiv.size());
  if (!gt_chunks.empty()) {
    // group sums: test g's sum lands in virtual set indiv_vbase + n_direct + g (the
    // group-tested requests' own slots, unused under group sums; a pass never has more
    // tests than group-tested requests), paired before k_group_coop
    GroupSums sums_fn;
    if (gsums)
      sums_fn = [&](const std::vector<uint32_t>& goff, const std::vector<uint32_t>& gmem) -> int {
        const uint32_t T = (uint32_t)(goff.size() - 1);
        if (n_direct + T > indiv.size()) return 1;
        std::vector<uint32_t> reqs(gmem.size());
        for (size_t k = 0; k < gmem.size(); ++k) reqs[k] = indiv[gmem[k]];
        GsumPlan gp;
        plan_gsum(in, goff, reqs, gp);
        if (gp.gsets.size() > n || gp.seg.size() > gseg_cap || (gp.level_off.size() > 1 && gp.level_off[1] > gtmp_cap))
          return 1;
        stage_copy(ctx, gsets_dev, gp.gsets.data(), sizeof(uint32_t) * gp.gsets.size());  // the stream is idle
        stage_copy(ctx, gseg_dev, gp.seg.data(), sizeof(uint32_t) * gp.seg.size());
        if (launch_gsum(ctx, b, gp, gseg_dev, gsets_dev, gtmp, indiv_vbase + n_direct, s)) return -1;
        HIPC(ctx, launch_ml_alone(indiv_vbase + n_direct, T, nullptr)); dbg_sync(s, "k_mln group sums");
        return 0;
      };
    gbufs.ref_fe = chunk_fe_kept ? b.chunk_fe : nullptr;
    if (const int rc = verify_groups(ctx, b, gbufs, gt_chunks, indiv_verdict, s, grp_cap, grp_mem_cap,
                                     gsums ? &sums_fn : nullptr))
      return rc;
    HIPC(ctx, hipEventRecord(ctx->ev[8], s));
    HIPC(ctx, hipEventRecord(ctx->ev1, s));
    HIPC(ctx, pass_wait(ctx, s));
  }
  assemble_verdicts(in, plan, chunk_ok.data(), indiv, indiv_verdict.data(), verdicts, stats);
  if (stats) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
    stats->device_ms = ms;
    // stage_ms: h2d, pk, pre, pset, exact, (unused), status+chunk, indiv
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

int bls_gpu_verify(bls_gpu_ctx* ctx, const bls_batch* in, int32_t* verdicts, bls_stats* stats) {
  return verify_impl(ctx, in, verdicts, stats, 0u, nullptr, nullptr);
}

int bls_gpu_verify_many(bls_gpu_ctx* ctx, const bls_batch* batches, uint32_t n_batches, int32_t* verdicts,
                        bls_stats* stats) {
  if (!ctx || (n_batches && (!batches || !verdicts))) return -2;
  if (stats) memset(stats, 0, sizeof(*stats));
  if (n_batches == 0) return 0;
  if (n_batches == 1) return verify_impl(ctx, batches, verdicts, stats, 0u, nullptr, nullptr);
  // messages with raw pubkeys keep their own pass: deserializeSet rejects a whole
  // message (worker.ts:43-46), which the merged pass does not track per message
  bool merge = true;
  for (uint32_t k = 0; k < n_batches; ++k) merge = merge && batches[k].set_pk_offsets != nullptr;
  if (!merge) {
    uint32_t off = 0;
    for (uint32_t k = 0; k < n_batches; ++k) {
      bls_stats st;
      const int rc = verify_impl(ctx, &batches[k], verdicts + off, stats ? &st : nullptr, 0u, nullptr, nullptr);
      if (rc != 0) return rc;
      off += batches[k].n_reqs;
      if (stats) {
        stats->batch_retries += st.batch_retries;
        stats->batch_sigs_success += st.batch_sigs_success;
        stats->n_chunks += st.n_chunks;
        stats->n_individual += st.n_individual;
        stats->n_flagged += st.n_flagged;
        stats->n_unique_msgs += st.n_unique_msgs;
        stats->n_ml_units += st.n_ml_units;
        stats->pass_shape |= st.pass_shape;
        stats->device_ms += st.device_ms;
      }
    }
    return 0;
  }
  // one pass over the concatenated messages (SoA arrays joined, offsets rebased); each
  // message passes verify_impl's shape checks before anything is read through it
  uint32_t n = 0, R = 0, n_idx = 0;
  bool lens = false;
  for (uint32_t k = 0; k < n_batches; ++k) {
    const bls_batch& b = batches[k];
    char what[32];
    snprintf(what, sizeof(what), "batch %u", k);
    if (const int rc = check_batch(ctx, &b, what)) return rc;
    if (b.n_reqs == 0 && b.n_sets != 0) {
      snprintf(ctx->err, sizeof(ctx->err), "%s: sets without requests", what);
      return -2;
    }
    n += b.n_sets;
    R += b.n_reqs;
    n_idx += b.set_pk_offsets[b.n_sets];
    lens = lens || b.signature_lens != nullptr;
  }
  std::vector<uint32_t> req_off(R + 1, 0), set_pk_off(n + 1, 0), pk_idx(n_idx ? n_idx : 1), sig_lens(lens ? n : 0);
  std::vector<uint8_t> batchable(R ? R : 1), msgs(32ull * n), sigs(96ull * n);
  std::vector<uint32_t> req_bounds(1, 0);
  uint32_t so = 0, ro = 0, io = 0;
  for (uint32_t k = 0; k < n_batches; ++k) {
    const bls_batch& b = batches[k];
    for (uint32_t r = 0; r < b.n_reqs; ++r) {
      req_off[ro + r + 1] = so + b.req_set_offsets[r + 1];
      batchable[ro + r] = b.req_batchable ? b.req_batchable[r] : 0;
    }
    for (uint32_t i = 0; i < b.n_sets; ++i) set_pk_off[so + i + 1] = io + b.set_pk_offsets[i + 1];
    if (b.set_pk_offsets[b.n_sets]) memcpy(&pk_idx[io], b.pk_indices, sizeof(uint32_t) * b.set_pk_offsets[b.n_sets]);
    if (b.n_sets) {
      memcpy(&msgs[32ull * so], b.messages, 32ull * b.n_sets);
      memcpy(&sigs[96ull * so], b.signatures, 96ull * b.n_sets);
    }
    for (uint32_t i = 0; lens && i < b.n_sets; ++i) sig_lens[so + i] = b.signature_lens ? b.signature_lens[i] : 96u;
    so += b.n_sets;
    ro += b.n_reqs;
    io += b.set_pk_offsets[b.n_sets];
    req_bounds.push_back(ro);
  }
  bls_batch all;
  memset(&all, 0, sizeof(all));
  all.n_sets = n;
  all.n_reqs = R;
  all.req_set_offsets = req_off.data();
  all.req_batchable = batchable.data();
  all.set_pk_offsets = set_pk_off.data();
  all.pk_indices = pk_idx.data();
  all.messages = msgs.data();
  all.signatures = sigs.data();
  all.signature_lens = lens ? sig_lens.data() : nullptr;
  all.seed = batches[0].seed;  // scalars: one random batch per pass (verdicts do not depend on them)
  return verify_impl(ctx, &all, verdicts, stats, 0u, nullptr, nullptr, nullptr, &req_bounds);
}

int bls_gpu_partial(bls_gpu_ctx* ctx, const bls_batch* in, uint32_t set_index_base, uint8_t* out576,
                    int32_t* status, uint32_t* err_info, bls_stats* stats) {
  if (!in || !out576 || !status) return -2;
  if (in->seed == nullptr) {
    snprintf(ctx->err, sizeof(ctx->err), "bls_gpu_partial needs the call's shared seed");
    return -2;
  }
  static_assert(sizeof(Fp12) == 576, "Fp12 wire size");
  if (in->n_sets == 0 || in->n_reqs == 0) {
    snprintf(ctx->err, sizeof(ctx->err), "bls_gpu_partial: empty shard");
    return -2;
  }
  memset(out576, 0, 576);
  if (err_info) err_info[0] = 3, err_info[1] = 0;
  return verify_impl(ctx, in, nullptr, stats, set_index_base, out576, status, err_info);
}

int bls_gpu_final_check(bls_gpu_ctx* ctx, const uint8_t* partials, uint32_t n, int32_t* verdict) {
  CTX_LOCK(ctx);
  HIPC(ctx, hipSetDevice(ctx->device));
  if (!partials || !verdict || n == 0) return -2;
  const uint32_t lvl1 = (n + FPROD_FAN - 1) / FPROD_FAN;
  Carver c{nullptr, 0};
  c.take<Fp12>(n);
  c.take<Fp12>(lvl1);
  c.take<Fp12>(lvl1);
  c.take<int32_t>(1);
  if (ensure_dev(ctx, c.off)) return -1;
  Carver d{ctx->dev_ws, 0};
  Fp12* in = d.take<Fp12>(n);
  Fp12* t[2] = {d.take<Fp12>(lvl1), d.take<Fp12>(lvl1)};
  int32_t* dv = d.take<int32_t>(1);
  hipStream_t s = ctx->stream;
  HIPC(ctx, hipMemcpyAsync(in, partials, 576ull * n, hipMemcpyHostToDevice, s));
  const Fp12* cur = in;
  uint32_t m = n, lvl = 0;
  while (m > FPROD_FAN) {
    HIPC(ctx, launch_k_fprod(cur, m, t[lvl & 1], nullptr, ctx->coop, s));
    cur = t[lvl & 1];
    m = (m + FPROD_FAN - 1) / FPROD_FAN;
    ++lvl;
  }
  HIPC(ctx, launch_k_fprod(cur, m, nullptr, dv, ctx->coop, s));
  HIPC(ctx, hipMemcpyAsync(verdict, dv, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipStreamSynchronize(s));
  return 0;
}

int bls_gpu_aggregate_pubkeys(bls_gpu_ctx* ctx, const uint32_t* set_pk_offsets, const uint32_t* pk_indices,
                              uint32_t n_sets, uint8_t* out96, int32_t* codes) {
  CTX_LOCK(ctx);
  HIPC(ctx, hipSetDevice(ctx->device));
  if (n_sets == 0) return 0;
  uint32_t n_idx = set_pk_offsets[n_sets];
  std::vector<uint32_t> agg_list;
  for (uint32_t i = 0; i < n_sets; ++i)
    if (set_pk_offsets[i + 1] - set_pk_offsets[i] >= BLS_AGG_WAVE_MIN) agg_list.push_back(i);
  PipeBufs b;
  memset(&b, 0, sizeof(b));
  auto carve = [&](Carver& c, uint8_t*& d_out) {
    b.set_pk_off = c.take<uint32_t>(n_sets + 1);
    b.pk_idx = c.take<uint32_t>(n_idx);
    b.agg_sets = c.take<uint32_t>(agg_list.size());
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
  b.n_agg = (uint32_t)agg_list.size();
  b.agg_min = agg_list.empty() ? 0u : BLS_AGG_WAVE_MIN;
  if (!agg_list.empty()) {
    HIPC(ctx, hipMemcpyAsync((void*)b.agg_sets, agg_list.data(), sizeof(uint32_t) * agg_list.size(),
                             hipMemcpyHostToDevice, s));
    HIPC(ctx, launch_k_pk_agg(b, s));  // the big aggregates first; k_aggregate serializes every set
  }
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

int bls_gpu_aggregate_signatures(bls_gpu_ctx* ctx, const uint8_t* sigs96, const uint32_t* list_offsets,
                                 uint32_t n_lists, uint8_t* out96, int32_t* codes) {
  CTX_LOCK(ctx);
  HIPC(ctx, hipSetDevice(ctx->device));
  if (n_lists == 0) return 0;
  if (!list_offsets || !out96 || !codes) return -2;
  const uint32_t n = list_offsets[n_lists];
  if (list_offsets[0] != 0) return -2;
  for (uint32_t l = 0; l < n_lists; ++l)
    if (list_offsets[l] > list_offsets[l + 1]) {
      snprintf(ctx->err, sizeof(ctx->err), "list_offsets not monotone at %u", l);
      return -2;
    }
  if (n > 0 && !sigs96) return -2;
  auto carve = [&](Carver& c, uint8_t*& d_in, uint32_t*& d_off, G2A*& d_pts, int32_t*& d_sc, uint8_t*& d_out,
                   int32_t*& d_codes) {
    d_in = c.take<uint8_t>(96ull * n);
    d_off = c.take<uint32_t>(n_lists + 1);
    d_pts = c.take<G2A>(n);
    d_sc = c.take<int32_t>(n);
    d_out = c.take<uint8_t>(96ull * n_lists);
    d_codes = c.take<int32_t>(n_lists);
  };
  uint8_t *d_in, *d_out;
  uint32_t* d_off;
  G2A* d_pts;
  int32_t *d_sc, *d_codes;
  {
    Carver c{nullptr, 0};
    carve(c, d_in, d_off, d_pts, d_sc, d_out, d_codes);
    if (ensure_dev(ctx, c.off)) return -1;
  }
  Carver c{ctx->dev_ws, 0};
  carve(c, d_in, d_off, d_pts, d_sc, d_out, d_codes);
  hipStream_t s = ctx->stream;
  if (n) HIPC(ctx, hipMemcpyAsync(d_in, sigs96, 96ull * n, hipMemcpyHostToDevice, s));
  HIPC(ctx, hipMemcpyAsync(d_off, list_offsets, sizeof(uint32_t) * (n_lists + 1), hipMemcpyHostToDevice, s));
  HIPC(ctx, launch_k_sig_aggregate(d_in, n, d_off, n_lists, d_pts, d_sc, d_out, d_codes, s));
  HIPC(ctx, hipMemcpyAsync(out96, d_out, 96ull * n_lists, hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipMemcpyAsync(codes, d_codes, sizeof(int32_t) * n_lists, hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipStreamSynchronize(s));
  return 0;
}

int bls_gpu_g2_decompress(bls_gpu_ctx* ctx, const uint8_t* in96, uint32_t n, int validate, uint8_t* out192,
                          int32_t* codes) {
  CTX_LOCK(ctx);
  HIPC(ctx, hipSetDevice(ctx->device));
  if (n == 0) return 0;
  if (!in96 || !out192 || !codes) return -2;
  Carver cv{nullptr, 0};
  cv.take<uint8_t>(96ull * n);
  cv.take<uint8_t>(192ull * n);
  cv.take<int32_t>(n);
  if (ensure_dev(ctx, cv.off)) return -1;
  Carver c{ctx->dev_ws, 0};
  uint8_t* d_in = c.take<uint8_t>(96ull * n);
  uint8_t* d_out = c.take<uint8_t>(192ull * n);
  int32_t* d_codes = c.take<int32_t>(n);
  hipStream_t s = ctx->stream;
  HIPC(ctx, hipMemcpyAsync(d_in, in96, 96ull * n, hipMemcpyHostToDevice, s));
  HIPC(ctx, launch_k_g2_decompress(d_in, n, validate, d_out, d_codes, s));
  HIPC(ctx, hipMemcpyAsync(out192, d_out, 192ull * n, hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipMemcpyAsync(codes, d_codes, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipStreamSynchronize(s));
  return 0;
}

int bls_gpu_ssz_roots(bls_gpu_ctx* ctx, uint32_t kind, const uint8_t* objs, uint32_t n, const uint8_t* domains,
                      uint32_t domain_stride, uint8_t* out32) {
  CTX_LOCK(ctx);
  if (!ssz_kind_known(kind) || (domains && domain_stride != 0 && domain_stride != 32)) {
    snprintf(ctx->err, sizeof(ctx->err), "bls_gpu_ssz_roots: unknown kind 0x%x or domain stride %u", kind,
             domain_stride);
    return -2;
  }
  HIPC(ctx, hipSetDevice(ctx->device));
  if (n == 0) return 0;
  if (!objs || !out32) return -2;
  const size_t obj_bytes = (size_t)BLS_SSZ_SIZE(kind) * n, dom_bytes = domains ? (domain_stride ? 32ull * n : 32) : 0;
  Carver cv{nullptr, 0};
  cv.take<uint8_t>(obj_bytes);
  cv.take<uint8_t>(dom_bytes);
  cv.take<uint8_t>(32ull * n);
  if (ensure_dev(ctx, cv.off)) return -1;
  Carver c{ctx->dev_ws, 0};
  uint8_t* d_obj = c.take<uint8_t>(obj_bytes);
  uint8_t* d_dom = c.take<uint8_t>(dom_bytes);
  uint8_t* d_out = c.take<uint8_t>(32ull * n);
  hipStream_t s = ctx->stream;
  HIPC(ctx, hipMemcpyAsync(d_obj, objs, obj_bytes, hipMemcpyHostToDevice, s));
  if (domains) HIPC(ctx, hipMemcpyAsync(d_dom, domains, dom_bytes, hipMemcpyHostToDevice, s));
  HIPC(ctx, launch_k_ssz_roots(kind, d_obj, n, domains ? d_dom : nullptr, domain_stride, d_out, s));
  HIPC(ctx, hipMemcpyAsync(out32, d_out, 32ull * n, hipMemcpyDeviceToHost, s));
  HIPC(ctx, hipStreamSynchronize(s));
  return 0;
}

int bls_gpu_hash_to_g2(bls_gpu_ctx* ctx, const uint8_t* msgs, uint32_t n, uint8_t* out192) {
  CTX_LOCK(ctx);
  return run_simple(ctx, n, 32, msgs, 0, nullptr, 192, out192, 0);
}

int bls_gpu_sk_to_pk(bls_gpu_ctx* ctx, const uint8_t* sks, uint32_t n, uint8_t* out48) {
  CTX_LOCK(ctx);
  return run_simple(ctx, n, 32, sks, 0, nullptr, 48, out48, 1);
}

int bls_gpu_sign(bls_gpu_ctx* ctx, const uint8_t* sks, const uint8_t* msgs, uint32_t n, uint8_t* out96) {
  CTX_LOCK(ctx);
  return run_simple(ctx, n, 32, sks, 32, msgs, 96, out96, 2);
}

}  // extern "C"

extern "C" int bls_gpu_set_debug_flags(bls_gpu_ctx* ctx, uint32_t flags) {
  if (!ctx) return -1;
  ctx->debug_flags = flags;
  return 0;
}

extern "C" int bls_gpu_mad_peak(bls_gpu_ctx* ctx, double* mads_per_s, double* ms_out) {
  CTX_LOCK(ctx);
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
  CTX_LOCK(ctx);
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
  CTX_LOCK(ctx);
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

extern "C" int bls_gpu_kernel_probe(bls_gpu_ctx* ctx, const char* name, uint32_t lanes, uint32_t reps, double* ms) {
  CTX_LOCK(ctx);
  HIPC(ctx, hipSetDevice(ctx->device));
  const size_t per = name ? kernel_probe_out_bytes(name) : 0;
  if (!per || !ms || lanes == 0) {
    snprintf(ctx->err, sizeof(ctx->err), "unknown probe %s", name ? name : "(null)");
    return -2;
  }
  if (ensure_dev(ctx, per * lanes)) return -1;
  hipStream_t s = ctx->stream;
  HIPC(ctx, launch_kernel_probe(name, ctx->dev_ws, lanes, s));  // warm-up
  HIPC(ctx, hipEventRecord(ctx->ev0, s));
  for (uint32_t r = 0; r < reps; ++r) HIPC(ctx, launch_kernel_probe(name, ctx->dev_ws, lanes, s));
  HIPC(ctx, hipEventRecord(ctx->ev1, s));
  HIPC(ctx, hipStreamSynchronize(s));
  float t = 0.f;
  HIPC(ctx, hipEventElapsedTime(&t, ctx->ev0, ctx->ev1));
  *ms = t;
  return 0;
}

// Probe: time the cooperative program `name` (blocks x reps runs); us_per_step is the
// wall time of one run divided by its step count.
extern "C" int bls_gpu_coop_probe(bls_gpu_ctx* ctx, const char* name, uint32_t blocks, uint32_t reps,
                                  double* us_per_step, double* ms_total, uint64_t* step_stamps) {
  CTX_LOCK(ctx);
  HIPC(ctx, hipSetDevice(ctx->device));
  CoopProg pg{0, 0};
  bool found = false;
  for (auto& e : *ctx->coop_progs)
    if (e.first == name) {
      pg = e.second;
      found = true;
    }
  if (!found) {
    snprintf(ctx->err, sizeof(ctx->err), "no program %s", name);
    return -1;
  }
  size_t sink_bytes = (4ull * blocks + 255) & ~(size_t)255;
  if (ensure_dev(ctx, sink_bytes + 8ull * (2 * pg.n + 1))) return -1;
  hipStream_t s = ctx->stream;
  uint64_t* d_stamps = (uint64_t*)(ctx->dev_ws + sink_bytes);
  HIPC(ctx, launch_k_coop_probe(ctx->coop, pg, blocks, 1, (uint32_t*)ctx->dev_ws, nullptr, s));
  HIPC(ctx, hipEventRecord(ctx->ev0, s));
  HIPC(ctx, launch_k_coop_probe(ctx->coop, pg, blocks, reps, (uint32_t*)ctx->dev_ws, nullptr, s));
  HIPC(ctx, hipEventRecord(ctx->ev1, s));
  HIPC(ctx, hipStreamSynchronize(s));
  float ms = 0.f;
  HIPC(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  *us_per_step = ms * 1e3 / ((double)reps * pg.n);
  if (ms_total) *ms_total = ms;
  if (step_stamps) {  // one more run of block 0 with s_memtime stamps: step start, compute done
    // (or the point $BLS_COOP_PROBE_MARK names, coop.hpp coop_step; steps that do not
    // reach it keep 0)
    const char* me = getenv("BLS_COOP_PROBE_MARK");
    const uint64_t mark = me ? strtoull(me, nullptr, 10) : 0ull;
    HIPC(ctx, hipMemsetAsync(d_stamps, 0, 8ull * (2 * pg.n + 1), s));
    HIPC(ctx, hipMemcpyAsync(d_stamps, &mark, 8, hipMemcpyHostToDevice, s));
    HIPC(ctx, hipStreamSynchronize(s));
    HIPC(ctx, launch_k_coop_probe(ctx->coop, pg, 1, 0, (uint32_t*)ctx->dev_ws, d_stamps, s));
    HIPC(ctx, hipMemcpyAsync(step_stamps, d_stamps, 8ull * (2 * pg.n + 1), hipMemcpyDeviceToHost, s));
    HIPC(ctx, hipStreamSynchronize(s));
  }
  return 0;
}
