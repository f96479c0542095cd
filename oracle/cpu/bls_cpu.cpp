// CPU BASELINE -- benchmark / test infrastructure only.  Never linked into the product
// library, never on the product path; bench.py's cpu_baseline leg and tests/ load it.
//
// A C++ restatement of the reference's CPU verify path, "not blst": Lodestar's
// BlsMultiThreadWorkerPool runs @chainsafe/blst on worker_threads
// (beacon-node/src/chain/bls/multithread/index.ts:98-423, worker.ts:32-108); blst is
// absent from /root/reference (yarn.lock:445-451), so this file restates the same
// structure on the host cores:
//   * one OS thread per worker (poolSize = cores, multithread/poolSize.ts:3-11);
//   * a worker message = verifyManySignatureSets(BlsWorkReq[]) (worker.ts:32-108):
//     deserializeSet over every request first (worker.ts:43-46), batchable requests
//     chunked by chunkifyMaximizeChunkSize(reqs, 16) (worker.ts:17,56), one
//     random-scalar batch per chunk, a failing / throwing chunk re-verified request
//     by request (worker.ts:76-98);
//   * verifySignatureSetsMaybeBatch (maybeBatch.ts:16-39): >= 2 sets ->
//     verifyMultipleSignatures with blst's structure [ext]: per set
//     Signature.fromBytes(sig, affine, validate=true) (decompress + G2 membership),
//     hash_to_G2, a non-zero 64-bit scalar r_i on both sides (r_i pk_i into the
//     Miller loop, r_i sig_i into an aggregate), then ONE Miller loop for
//     (-g1, sum r_i sig_i) and one final exponentiation; Miller loops run 8 pairs at a
//     time with the f squarings shared (blst's miller_loop_n, N_MAX = 8);
//     1 set -> e(pk, H(m)) == e(g1, sig) (Signature.verify).
// The field arithmetic is the kernels' __host__ __device__ code compiled for the CPU
// (lodestar_amd/csrc/bls/*.hpp, host path: 6 x 64-bit words, unsigned __int128 CIOS).
//
// Build: oracle/cpu/Makefile (g++ -O3 -std=c++17 -pthread, shared library).
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "bls/hash_to_curve.hpp"
#include "bls/pairing.hpp"
#include "bls/pipeline.hpp"

unsigned long long bls_fpm_counter = 0;

using namespace bls;

namespace {

struct DSet {
  G1A pk;
  const uint8_t* msg;
  const uint8_t* sig;
  uint32_t sig_len;
};

// prod_k f_{|x|,Q_k}(P_k) with shared squarings (blst miller_loop_n), conjugated
Fp12 miller_loop_n(const G1Eval* P, const G2A* Q, int n) {
  G2Proj T[8];
  for (int k = 0; k < n; ++k) {
    T[k].x = Q[k].x;
    T[k].y = Q[k].y;
    T[k].z = fp2_one();
  }
  Fp12 f = fp12_one();
  Fp2 c0, c1, c2;
  const uint64_t X = BLS_X_ABS;
  for (int i = 62; i >= 0; --i) {
    if (i != 62) f = fp12_sqr(f);
    for (int k = 0; k < n; ++k) {
      miller_dbl_step(T[k], c0, c1, c2);
      f = line_mul(f, P[k], c0, c1, c2);
    }
    if ((X >> i) & 1ull) {
      for (int k = 0; k < n; ++k) {
        miller_add_step(T[k], Q[k], c0, c1, c2);
        f = line_mul(f, P[k], c0, c1, c2);
      }
    }
  }
  return fp12_conj(f);
}

// accumulate pairs 8 at a time into f
struct PairAcc {
  G1Eval P[8];
  G2A Q[8];
  int n = 0;
  Fp12 f = fp12_one();
  void add(const G1Eval& p, const G2A& q) {
    P[n] = p;
    Q[n] = q;
    if (++n == 8) flush();
  }
  void flush() {
    if (n) f = fp12_mul(f, miller_loop_n(P, Q, n));
    n = 0;
  }
};

uint64_t next_scalar(uint64_t& state) {  // splitmix64, forced non-zero (randomBytesNonZero(8))
  uint64_t z = (state += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  return z ? z : 1;
}

int32_t decode_sig(const DSet& s, G2A& sig) {
  if (s.sig_len != 96) return BLS_INVALID_SIZE;
  int32_t code = g2_decompress96(s.sig, sig);
  if (code == BLS_OK && !sig.inf && !g2_in_subgroup(sig)) code = BLS_POINT_NOT_IN_GROUP;
  return code;
}

// verifySignatureSetsMaybeBatch (maybeBatch.ts:16-39): 1 / 0, or -code when it throws
int32_t maybe_batch(const DSet* sets, uint32_t n, uint64_t& rng) {
  if (n == 0) return -BLS_EMPTY_SET;
  std::vector<G2A> sigs(n);
  for (uint32_t i = 0; i < n; ++i) {
    int32_t code = decode_sig(sets[i], sigs[i]);
    if (code != BLS_OK) return -code;
  }
  if (n == 1) {  // Signature.verify: e(pk, H(m)) * e(-g1, sig) == 1
    if (sigs[0].inf) return -BLS_ZERO_SIGNATURE;
    if (sets[0].pk.inf) return -BLS_PK_IS_INFINITY;
    uint32_t w[8];
    msg_words_from_bytes(sets[0].msg, w);
    PairAcc acc;
    acc.add(g1_eval_from_aff(sets[0].pk), hash_to_g2(w));
    acc.add(neg_g1_eval(), sigs[0]);
    acc.flush();
    return fp12_is_one(final_exponentiation(acc.f)) ? 1 : 0;
  }
  PairAcc acc;
  G2J agg = jac_infinity<Fp2>();
  for (uint32_t i = 0; i < n; ++i) {
    if (sets[i].pk.inf) return -BLS_PK_IS_INFINITY;
    const uint64_t r = next_scalar(rng);
    uint32_t w[8];
    msg_words_from_bytes(sets[i].msg, w);
    const G1J rpk = jac_mul_u64(jac_from_aff(sets[i].pk), r);
    acc.add(g1_eval_from_jac(rpk), hash_to_g2(w));
    if (!sigs[i].inf) agg = jac_add(agg, aff_mul_u64(sigs[i], r));
  }
  if (!jac_is_inf(agg)) acc.add(neg_g1_eval(), jac_to_aff(agg));
  acc.flush();
  return fp12_is_one(final_exponentiation(acc.f)) ? 1 : 0;
}

}  // namespace

extern "C" {

// verifyManySignatureSets (worker.ts:32-108) over one bls_batch with raw 96-byte keys
// (the worker wire format, index.ts:126,160).  verdicts: n_reqs (1 / 0 / -code).
// Returns 0, or -1 when a key does not decode (the whole message rejects:
// worker.ts:45 throws, index.ts:367-374), every verdict then holding that code.
int cpu_verify_many(const bls_batch* in, int32_t* verdicts, uint32_t* batch_retries, uint32_t* batch_sigs_success,
                    uint64_t seed) {
  const uint32_t R = in->n_reqs;
  std::vector<DSet> sets(in->n_sets);
  for (uint32_t i = 0; i < in->n_sets; ++i) {  // deserializeSet, every request first
    int32_t code = g1_deserialize96(in->pubkeys + 96ull * i, sets[i].pk);
    if (code != BLS_OK) {
      for (uint32_t r = 0; r < R; ++r) verdicts[r] = -code;
      return -1;
    }
    sets[i].msg = in->messages + 32ull * i;
    sets[i].sig = in->signatures + 96ull * i;
    sets[i].sig_len = in->signature_lens ? in->signature_lens[i] : 96;
  }
  uint64_t rng = seed;
  BatchPlan plan;
  plan_batch(in, plan);
  std::vector<uint32_t> retry = plan.nonbatch_reqs;
  uint32_t retries = 0, ok_sigs = 0;
  for (size_t c = 0; c + 1 < plan.chunk_off.size(); ++c) {
    std::vector<DSet> all;
    for (uint32_t k = plan.chunk_off[c]; k < plan.chunk_off[c + 1]; ++k) {
      const uint32_t r = plan.chunk_reqs[k];
      for (uint32_t i = in->req_set_offsets[r]; i < in->req_set_offsets[r + 1]; ++i) all.push_back(sets[i]);
    }
    if (maybe_batch(all.data(), (uint32_t)all.size(), rng) == 1) {
      for (uint32_t k = plan.chunk_off[c]; k < plan.chunk_off[c + 1]; ++k) {
        const uint32_t r = plan.chunk_reqs[k];
        verdicts[r] = 1;
        ok_sigs += in->req_set_offsets[r + 1] - in->req_set_offsets[r];
      }
    } else {
      ++retries;
      for (uint32_t k = plan.chunk_off[c]; k < plan.chunk_off[c + 1]; ++k) retry.push_back(plan.chunk_reqs[k]);
    }
  }
  for (uint32_t r : retry) {
    const uint32_t beg = in->req_set_offsets[r], end = in->req_set_offsets[r + 1];
    verdicts[r] = maybe_batch(sets.data() + beg, end - beg, rng);
  }
  if (batch_retries) *batch_retries = retries;
  if (batch_sigs_success) *batch_sigs_success = ok_sigs;
  return 0;
}

// Worker-pool throughput: `threads` workers, each running verifyManySignatureSets on
// its own copy of `job` back to back until `seconds` have passed (every worker finishes
// the message it is in).  Returns sets/s = all verified sets / wall time; *messages =
// worker messages completed.  A message that does not verify all-valid returns -1.
int cpu_pool_throughput(const bls_batch* job, int threads, double seconds, double* sets_per_s, uint32_t* messages) {
  std::atomic<uint32_t> done{0};
  std::atomic<int> bad{0};
  const auto t0 = std::chrono::steady_clock::now();
  const auto stop = t0 + std::chrono::duration<double>(seconds);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t] {
      std::vector<int32_t> v(job->n_reqs);
      uint64_t seed = 0x1234567ull * (t + 1);
      do {
        cpu_verify_many(job, v.data(), nullptr, nullptr, seed++);
        for (int32_t x : v)
          if (x != 1) bad = 1;
        done++;
      } while (std::chrono::steady_clock::now() < stop);
    });
  }
  for (auto& th : pool) th.join();
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *messages = done.load();
  *sets_per_s = (double)done.load() * job->n_sets / dt;
  return bad ? -1 : 0;
}

// Latency of one worker message on one core: `runs` timed runs (ms each) after 2 warm-ups.
int cpu_message_latency(const bls_batch* job, int runs, double* ms) {
  std::vector<int32_t> v(job->n_reqs);
  for (int w = 0; w < 2; ++w) cpu_verify_many(job, v.data(), nullptr, nullptr, 7 + w);
  for (int k = 0; k < runs; ++k) {
    const auto t0 = std::chrono::steady_clock::now();
    cpu_verify_many(job, v.data(), nullptr, nullptr, 100 + k);
    ms[k] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (int32_t x : v)
      if (x != 1) return -1;
  }
  return 0;
}

}  // extern "C"
