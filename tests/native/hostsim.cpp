// TEST INFRASTRUCTURE ONLY -- never linked into the product library.
//
// Compiles the HIP kernels' __host__ __device__ math (lodestar_amd/csrc/bls/*.hpp)
// for the CPU so tests/ can check every device routine against the Python
// oracle (oracle/bls_oracle.py) without a GPU, and count Fp multiplications per
// stage (the algorithmic work model behind bench.py's roofline figure).
//
// All byte interfaces use canonical big-endian encodings:
//   Fp = 48 B; Fp2 = c0 || c1 (96 B); Fp12 = w-basis coefficients k = 0..5, each Fp2 (576 B);
//   G1 = 96 B uncompressed (x || y); G2 = 192 B uncompressed (ZCash order x.c1 x.c0 y.c1 y.c0).
#include <string.h>

// the device's exponentiation chains (field.hpp fp_pow_const -> lazy28.hpp lz_pow_const)
#define BLS_LAZY_POW 1
#include "bls/pairing.hpp"
#include "bls/hash_to_curve.hpp"
#include "bls/pipeline.hpp"
#include "bls/group_decode.hpp"

unsigned long long bls_fpm_counter = 0;
unsigned long long bls_lz_norm_counter = 0;

using namespace bls;

static Fp rd_fp(const uint8_t* b) { return fp_to_mont(fp_from_be48(b)); }
static void wr_fp(const Fp& a, uint8_t* b) { fp_to_be48(fp_from_mont(a), b); }
static Fp2 rd_fp2(const uint8_t* b) { return Fp2{rd_fp(b), rd_fp(b + 48)}; }
static void wr_fp2(const Fp2& a, uint8_t* b) {
  wr_fp(a.c0, b);
  wr_fp(a.c1, b + 48);
}
static Fp2* coef(Fp12& f, int k) {
  switch (k) {
    case 0: return &f.c0.c0;
    case 1: return &f.c1.c0;
    case 2: return &f.c0.c1;
    case 3: return &f.c1.c1;
    case 4: return &f.c0.c2;
    default: return &f.c1.c2;
  }
}
static Fp12 rd_fp12(const uint8_t* b) {
  Fp12 f;
  for (int k = 0; k < 6; ++k) *coef(f, k) = rd_fp2(b + 96 * k);
  return f;
}
static void wr_fp12(Fp12 f, uint8_t* b) {
  for (int k = 0; k < 6; ++k) wr_fp2(*coef(f, k), b + 96 * k);
}
static G1A rd_g1(const uint8_t* b) {
  G1A a;
  a.inf = (b[0] & 0x40) != 0;
  if (a.inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a.x = rd_fp(b);
    a.y = rd_fp(b + 48);
  }
  return a;
}
static G2A rd_g2(const uint8_t* b) {
  G2A a;
  a.inf = (b[0] & 0x40) != 0;
  if (a.inf) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    a.x = Fp2{rd_fp(b + 48), rd_fp(b)};
    a.y = Fp2{rd_fp(b + 144), rd_fp(b + 96)};
  }
  return a;
}

extern "C" {

// kernels/k_chain.hip's windowed [k]P (curve.hpp jac_mul_u64_w4) against
// double-and-add on multiples of the generators, for n scalars from a splitmix64
// stream plus the edge scalars; returns the number of mismatches
static uint64_t hs_splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
int hs_mul_window_check(unsigned long long seed, int n) {
  uint64_t st = seed;
  int bad = 0;
  const uint64_t edge[] = {0ull, 1ull, 15ull, 16ull, 0x0FFFFFFFFFFFFFFFull, 1ull << 60, 0xFFFFFFFFFFFFFFFFull,
                           0x8000000000000001ull};
  for (int i = 0; i < n + 8; ++i) {
    const uint64_t k = i < 8 ? edge[i] : hs_splitmix(st);
    const uint64_t m = hs_splitmix(st) | 1ull;
    G1J T1[15];
    const G1J p1 = jac_mul_u64(jac_from_aff(g1_generator()), m);
    if (!jac_eq(jac_mul_u64_w4<Fp>(p1, nullptr, k, T1), jac_mul_u64(p1, k))) ++bad;
    G2J T2[15];
    G2A a2 = g2_generator();
    if (i & 1) {  // an affine base other than the generator: [m] g2, normalised
      const G2J j2 = jac_mul_u64(jac_from_aff(a2), m);
      const Fp2 zi = fp2_inv(j2.z), zi2 = fp2_sqr(zi);
      a2.x = fp2_mul(j2.x, zi2);
      a2.y = fp2_mul(j2.y, fp2_mul(zi2, zi));
    }
    if (!jac_eq(jac_mul_u64_w4<Fp2>(jac_from_aff(a2), &a2, k, T2), aff_mul_u64(a2, k))) ++bad;
  }
  return bad;
}

// curve.hpp jac_mul_glv (k_chain's [r] pk / [r] sig): [a + b mu]P for the G1 / G2 base
// [m]g against [k]P by double-and-add over k = (a + b mu) mod r (k8: 8 little-endian
// words, computed by the test); 1 when equal
int hs_glv_check(uint32_t a, uint32_t b, const uint32_t* k8, uint64_t m, int g2) {
  if (!g2) {
    const G1A base = jac_to_aff(jac_mul_u64(jac_from_aff(g1_generator()), m));
    G1J T[15];
    return jac_eq(jac_mul_glv<Fp>(jac_from_aff(base), a, b, T), aff_mul_u256(base, k8)) ? 1 : 0;
  }
  const G2A base = jac_to_aff(jac_mul_u64(jac_from_aff(g2_generator()), m));
  G2J T[15];
  return jac_eq(jac_mul_glv<Fp2>(jac_from_aff(base), a, b, T), aff_mul_u256(base, k8)) ? 1 : 0;
}

unsigned long long hs_fpm_count(void) { return bls_fpm_counter; }
void hs_fpm_reset(void) { bls_fpm_counter = 0; }

void hs_fp_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { wr_fp(fp_mul(rd_fp(a), rd_fp(b)), out); }
// the device's 28-bit-digit Montgomery product on raw little-endian limbs (no
// Montgomery conversion): out = a * b / 2^384 mod p, lazy (< 2p) for inputs < 3p
void hs_fp_mul_d28_raw(const uint8_t* a, const uint8_t* b, uint8_t* out, int sqr) {
  Fp x, y;
  memcpy(x.l, a, 48);
  memcpy(y.l, b, 48);
  Fp r = sqr ? fp_sqr_d28_lazy(x) : fp_mul_d28_lazy(x, y);
  memcpy(out, r.l, 48);
}
void hs_fp_add(const uint8_t* a, const uint8_t* b, uint8_t* out) { wr_fp(fp_add(rd_fp(a), rd_fp(b)), out); }
void hs_fp_sub(const uint8_t* a, const uint8_t* b, uint8_t* out) { wr_fp(fp_sub(rd_fp(a), rd_fp(b)), out); }
void hs_fp_half(const uint8_t* a, uint8_t* out) { wr_fp(fp_half(rd_fp(a)), out); }
void hs_fp_inv(const uint8_t* a, uint8_t* out) { wr_fp(fp_inv(rd_fp(a)), out); }
void hs_fp_inv_gcd(const uint8_t* a, uint8_t* out) { wr_fp(fp_inv_gcd(rd_fp(a)), out); }
int hs_fp_sqrt(const uint8_t* a, uint8_t* out) {
  Fp r;
  bool ok = fp_sqrt(rd_fp(a), r);
  wr_fp(r, out);
  return ok;
}

void hs_fp2_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { wr_fp2(fp2_mul(rd_fp2(a), rd_fp2(b)), out); }
// field.hpp fp2_mul_s on raw limbs: coefficients < 2p (unreduced sums), canonical out
void hs_fp2_mul_s_raw(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  Fp2 x, y;
  memcpy(x.c0.l, a, 48);
  memcpy(x.c1.l, a + 48, 48);
  memcpy(y.c0.l, b, 48);
  memcpy(y.c1.l, b + 48, 48);
  const Fp2 r = fp2_mul_s(x, y);
  memcpy(out, r.c0.l, 48);
  memcpy(out + 48, r.c1.l, 48);
}
// the device's lazy Fp2 product (field.hpp fp2_mul_d28) on raw limbs (Montgomery form in, out)
void hs_fp2_mul_d28_raw(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  Fp a0, a1, b0, b1;
  memcpy(a0.l, a, 48);
  memcpy(a1.l, a + 48, 48);
  memcpy(b0.l, b, 48);
  memcpy(b1.l, b + 48, 48);
  const Fp2 r = fp2_mul_d28(a0, a1, b0, b1);
  memcpy(out, r.c0.l, 48);
  memcpy(out + 48, r.c1.l, 48);
}
void hs_fp2_sqr_d28_raw(const uint8_t* a, uint8_t* out) {
  Fp a0, a1;
  memcpy(a0.l, a, 48);
  memcpy(a1.l, a + 48, 48);
  const Fp2 r = fp2_sqr_d28(a0, a1);
  memcpy(out, r.c0.l, 48);
  memcpy(out + 48, r.c1.l, 48);
}
void hs_fp2_sqr(const uint8_t* a, uint8_t* out) { wr_fp2(fp2_sqr(rd_fp2(a)), out); }
void hs_fp2_inv(const uint8_t* a, uint8_t* out) { wr_fp2(fp2_inv(rd_fp2(a)), out); }
int hs_fp2_sqrt(const uint8_t* a, uint8_t* out) {
  Fp2 r = fp2_zero();
  bool ok = fp2_sqrt(rd_fp2(a), r);
  wr_fp2(r, out);
  return ok;
}
int hs_fp2_sgn0(const uint8_t* a) { return (int)fp2_sgn0(rd_fp2(a)); }

void hs_fp12_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { wr_fp12(fp12_mul(rd_fp12(a), rd_fp12(b)), out); }
void hs_fp12_sqr(const uint8_t* a, uint8_t* out) { wr_fp12(fp12_sqr(rd_fp12(a)), out); }
void hs_fp12_cyclotomic_sqr(const uint8_t* a, uint8_t* out) { wr_fp12(fp12_cyclotomic_sqr(rd_fp12(a)), out); }
void hs_fp12_inv(const uint8_t* a, uint8_t* out) { wr_fp12(fp12_inv(rd_fp12(a)), out); }
void hs_fp12_frob(const uint8_t* a, uint8_t* out) { wr_fp12(fp12_frob(rd_fp12(a)), out); }
void hs_fp12_frob2(const uint8_t* a, uint8_t* out) { wr_fp12(fp12_frob2(rd_fp12(a)), out); }
void hs_fp12_mul_line(const uint8_t* f, const uint8_t* l0, const uint8_t* l2, const uint8_t* l3, uint8_t* out) {
  wr_fp12(fp12_mul_line(rd_fp12(f), rd_fp2(l0), rd_fp2(l2), rd_fp2(l3)), out);
}
// one f over two lanes (k_mlf2): both halves' products, swapped, joined by each half;
// out: half 0's result then half 1's (576 bytes each)
void hs_fp12_sqr_pair(const uint8_t* a, uint8_t* out) {
  const Fp12 x = rd_fp12(a);
  const Fp6 m0 = fp12_sqr_half_prod(x, false), m1 = fp12_sqr_half_prod(x, true);
  wr_fp12(fp12_sqr_half_join(m0, m1, false), out);
  wr_fp12(fp12_sqr_half_join(m1, m0, true), out + 576);
}
void hs_fp12_mul_line_pair(const uint8_t* f, const uint8_t* l0, const uint8_t* l2, const uint8_t* l3, uint8_t* out) {
  const Fp12 x = rd_fp12(f);
  const Fp2 a = rd_fp2(l0), b = rd_fp2(l2), c = rd_fp2(l3);
  const LineHalf h0 = fp12_line_half_prod(x, a, b, c, false), h1 = fp12_line_half_prod(x, a, b, c, true);
  wr_fp12(fp12_line_half_join(h0, h1.m, h1.p, false), out);
  wr_fp12(fp12_line_half_join(h1, h0.m, h0.p, true), out + 576);
}
void hs_fp12_mul_line2(const uint8_t* f, const uint8_t* l, const uint8_t* m, uint8_t* out) {
  wr_fp12(fp12_mul_line2(rd_fp12(f), rd_fp2(l), rd_fp2(l + 96), rd_fp2(l + 192), rd_fp2(m), rd_fp2(m + 96),
                         rd_fp2(m + 192)),
          out);
}
void hs_final_exp(const uint8_t* a, uint8_t* out) { wr_fp12(final_exponentiation(rd_fp12(a)), out); }
// bls_gpu.hip verify_groups' decode of one failed chunk (bls/group_decode.hpp)
int hs_group_decode(uint32_t m, uint32_t nbits, int whole_pass, const int32_t* v) {
  return group_decode(m, nbits, whole_pass != 0, v);
}

void hs_miller_loop(const uint8_t* g1, const uint8_t* g2, uint8_t* out) {
  wr_fp12(miller_loop(g1_eval_from_aff(rd_g1(g1)), rd_g2(g2)), out);
}
// Miller loop with the G1 point given in Jacobian form (x z^2, y z^3, z) for a scaling z
void hs_miller_loop_jac(const uint8_t* g1, const uint8_t* z48, const uint8_t* g2, uint8_t* out) {
  G1A a = rd_g1(g1);
  Fp z = rd_fp(z48);
  G1J j;
  Fp z2 = fp_sqr(z);
  j.x = fp_mul(a.x, z2);
  j.y = fp_mul(a.y, fp_mul(z2, z));
  j.z = z;
  wr_fp12(miller_loop(g1_eval_from_jac(j), rd_g2(g2)), out);
}
void hs_pairing(const uint8_t* g1, const uint8_t* g2, uint8_t* out) {
  wr_fp12(final_exponentiation(miller_loop(g1_eval_from_aff(rd_g1(g1)), rd_g2(g2))), out);
}

void hs_hash_to_g2(const uint8_t* msg32, uint8_t* out192) {
  uint32_t w[8];
  msg_words_from_bytes(msg32, w);
  g2_serialize192(hash_to_g2(w), out192);
}
void hs_map_to_curve_sswu(const uint8_t* u96, uint8_t* out192) {
  G2A r = map_to_curve_sswu(rd_fp2(u96));
  wr_fp2(r.x, out192);
  wr_fp2(r.y, out192 + 96);
}
int hs_map_to_curve_sswu_fast(const uint8_t* u96, uint8_t* out192) {
  Fp2 x, y;
  if (!map_to_curve_sswu_fast(rd_fp2(u96), x, y)) return 0;
  wr_fp2(x, out192);
  wr_fp2(y, out192 + 96);
  return 1;
}
void hs_hash_to_field(const uint8_t* msg32, uint8_t* out384) {
  uint32_t w[8];
  msg_words_from_bytes(msg32, w);
  Fp2 u0, u1;
  hash_to_field_fp2_x2(w, u0, u1);
  wr_fp2(u0, out384);
  wr_fp2(u1, out384 + 96);
}
void hs_expand_message_xmd(const uint8_t* msg32, uint8_t* out256) {
  uint32_t w[8], o[64];
  msg_words_from_bytes(msg32, w);
  expand_message_xmd_32(w, o);
  for (int i = 0; i < 64; ++i) {
    out256[4 * i] = (uint8_t)(o[i] >> 24);
    out256[4 * i + 1] = (uint8_t)(o[i] >> 16);
    out256[4 * i + 2] = (uint8_t)(o[i] >> 8);
    out256[4 * i + 3] = (uint8_t)o[i];
  }
}

int hs_g2_decompress(const uint8_t* sig96, uint8_t* out192) {
  G2A a;
  int32_t code = g2_decompress96(sig96, a);
  if (code == BLS_OK) g2_serialize192(a, out192);
  return code;
}
int hs_g2_in_subgroup(const uint8_t* g2) { return g2_in_subgroup(rd_g2(g2)); }
int hs_g1_decompress(const uint8_t* pk48, uint8_t* out96) {
  G1A a;
  int32_t code = g1_decompress48(pk48, a);
  if (code == BLS_OK) g1_serialize96(a, out96);
  return code;
}
void hs_g2_compress(const uint8_t* g2, uint8_t* out96) { g2_compress96(rd_g2(g2), out96); }
void hs_g1_compress(const uint8_t* g1, uint8_t* out48) { g1_compress48(rd_g1(g1), out48); }
// the aggregated-signature path's Jacobian isogeny (k_chain role 0), as an affine point;
// returns 0 for the point at infinity
int hs_iso_map_jac(const uint8_t* xy192, uint8_t* out192) {
  const G2J r = iso_map_jac(rd_fp2(xy192), rd_fp2(xy192 + 96));
  if (jac_is_inf(r)) return 0;
  const G2A a = jac_to_aff(r);
  wr_fp2(a.x, out192);
  wr_fp2(a.y, out192 + 96);
  return 1;
}
void hs_g2_clear_cofactor(const uint8_t* g2, uint8_t* out192) {
  g2_serialize192(jac_to_aff(g2_clear_cofactor(jac_from_aff(rd_g2(g2)))), out192);
}
void hs_g1_mul_u64(const uint8_t* g1, uint64_t k, uint8_t* out96) {
  g1_serialize96(jac_to_aff(aff_mul_u64(rd_g1(g1), k)), out96);
}
void hs_g2_mul_u64(const uint8_t* g2, uint64_t k, uint8_t* out192) {
  g2_serialize192(jac_to_aff(aff_mul_u64(rd_g2(g2), k)), out192);
}
void hs_g1_add(const uint8_t* a, const uint8_t* b, uint8_t* out96) {
  g1_serialize96(jac_to_aff(jac_add(jac_from_aff(rd_g1(a)), jac_from_aff(rd_g1(b)))), out96);
}
void hs_g2_add(const uint8_t* a, const uint8_t* b, uint8_t* out192) {
  g2_serialize192(jac_to_aff(jac_add(jac_from_aff(rd_g2(a)), jac_from_aff(rd_g2(b)))), out192);
}
void hs_g2_dbl(const uint8_t* a, uint8_t* out192) {
  g2_serialize192(jac_to_aff(jac_dbl(jac_from_aff(rd_g2(a)))), out192);
}

// sk: 32 bytes big-endian
void hs_sk_to_pk(const uint8_t* sk, uint8_t* out48) {
  uint32_t k[8];
  scalar_words_from_be32(sk, k);
  g1_compress48(jac_to_aff(aff_mul_u256(g1_generator(), k)), out48);
}
void hs_sign(const uint8_t* sk, const uint8_t* msg32, uint8_t* out96) {
  uint32_t k[8], w[8];
  scalar_words_from_be32(sk, k);
  msg_words_from_bytes(msg32, w);
  g2_compress96(jac_to_aff(aff_mul_u256(hash_to_g2(w), k)), out96);
}

}  // extern "C"

#include <vector>

static std::vector<G1A> g_table;
// Fp multiplications per stage of the last hs_verify_batch:
// pk, sig, h2c, scale, miller, status+chunk, individual
static unsigned long long g_stage_fpm[7];

extern "C" {

unsigned long long hs_stage_fpm(int k) { return (k >= 0 && k < 7) ? g_stage_fpm[k] : 0ull; }

// Pubkey table for the host pipeline (mirrors bls_gpu_load_pubkeys)
long long hs_load_pubkeys(const uint8_t* pks, uint32_t n, uint32_t pk_len, int32_t* codes) {
  for (uint32_t i = 0; i < n; ++i) {
    G1A a;
    int32_t c = pk_len == 48 ? g1_decompress48(pks + 48ull * i, a) : g1_deserialize96(pks + 96ull * i, a);
    if (codes) codes[i] = c;
    if (c != BLS_OK) {
      a.inf = true;
      a.x = fp_zero();
      a.y = fp_zero();
    }
    g_table.push_back(a);
  }
  return (long long)g_table.size();
}
void hs_clear_pubkeys(void) { g_table.clear(); }

// Full verify pipeline on the CPU: the GPU kernels' stage bodies (pipeline.hpp) looped
// over "lanes", planned and assembled by the same host code as bls_gpu_verify.
int hs_verify_batch(const bls_batch* in, int32_t* verdicts, bls_stats* stats) {
  BatchPlan plan;
  plan_batch(in, plan);
  uint32_t n = in->n_sets, R = in->n_reqs;
  std::vector<G2A> sig(n), H(n);
  std::vector<G1J> pk(n), rpk(n);
  std::vector<G2J> rsig(n);
  std::vector<Fp12> f(n);
  std::vector<int32_t> sig_status(n), pk_status(n), req_status(R);
  uint32_t n_chunks = (uint32_t)plan.chunk_off.size() - 1;
  std::vector<int32_t> chunk_ok(n_chunks + 1);
  uint32_t seed[8];
  if (in->seed) {
    scalar_words_from_be32(in->seed, seed);
  } else {
    for (int k = 0; k < 8; ++k) seed[k] = 0x9e3779b9u * (k + 1);
  }
  PipeBufs b;
  memset(&b, 0, sizeof(b));
  b.n_sets = n;
  b.n_reqs = R;
  b.n_chunks = n_chunks;
  b.req_off = in->req_set_offsets;
  b.pubkeys = in->pubkeys;
  b.set_pk_off = in->set_pk_offsets;
  b.pk_idx = in->pk_indices;
  b.pk_table = g_table.data();
  b.pk_table_n = (uint32_t)g_table.size();
  b.msgs = in->messages;
  b.sigs = in->signatures;
  b.sig_lens = in->signature_lens;
  b.seed = seed;
  b.chunk_off = plan.chunk_off.data();
  b.chunk_reqs = plan.chunk_reqs.data();
  b.sig = sig.data();
  b.sig_status = sig_status.data();
  b.pk = pk.data();
  b.pk_status = pk_status.data();
  uint32_t first_bad_pk = 0xFFFFFFFFu;
  if (in->pubkeys && !in->set_pk_offsets) b.first_bad_pk = &first_bad_pk;
  b.H = H.data();
  b.rpk = rpk.data();
  b.rsig = rsig.data();
  b.f = f.data();
  b.req_status = req_status.data();
  b.chunk_ok = chunk_ok.data();
  unsigned long long c0 = bls_fpm_counter;
  auto mark = [&](int k) {
    g_stage_fpm[k] = bls_fpm_counter - c0;
    c0 = bls_fpm_counter;
  };
  for (uint32_t i = 0; i < n; ++i) stage_pk(b, i);
  mark(0);
  for (uint32_t i = 0; i < n; ++i) stage_sig(b, i);
  mark(1);
  for (uint32_t i = 0; i < n; ++i) stage_h2c(b, i);
  mark(2);
  for (uint32_t i = 0; i < n; ++i) stage_scale(b, i);
  mark(3);
  for (uint32_t i = 0; i < n; ++i) stage_pair_set(b, i);
  mark(4);
  for (uint32_t r = 0; r < R; ++r) stage_req_status(b, r);
  for (uint32_t c = 0; c < n_chunks; ++c) stage_chunk(b, c);
  mark(5);
  std::vector<uint32_t> indiv = plan.nonbatch_reqs;
  for (uint32_t c = 0; c < n_chunks; ++c)
    if (chunk_ok[c] != 1)
      for (uint32_t k = plan.chunk_off[c]; k < plan.chunk_off[c + 1]; ++k) indiv.push_back(plan.chunk_reqs[k]);
  std::vector<int32_t> indiv_verdict(indiv.size() + 1);
  b.indiv_reqs = indiv.data();
  b.n_indiv = (uint32_t)indiv.size();
  b.indiv_verdict = indiv_verdict.data();
  for (uint32_t t = 0; t < b.n_indiv; ++t) stage_indiv(b, t);
  mark(6);
  assemble_verdicts(in, plan, chunk_ok.data(), indiv, indiv_verdict.data(), verdicts, stats);
  return 0;
}

// Signing-root dedup: plan_msg_dedup + stage_pre (2u map lanes) + stage_qdup must
// leave every set with the SSWU points and flags the per-set pre-stage gives it.
// Returns n_uniq, or -1 on a mismatch (q_out gets the deduplicated points).
int hs_pre_dedup_check(const uint8_t* msgs, uint32_t n, uint32_t* uniq_out, uint32_t* rep_out, uint8_t* q_out) {
  std::vector<uint32_t> uniq, rep;
  const uint32_t u = plan_msg_dedup(msgs, n, uniq, rep);
  std::vector<uint8_t> sigs(96ull * n, 0);
  std::vector<uint32_t> lens(n, 0);
  std::vector<G2A> sig(n);
  std::vector<int32_t> sig_status(n);
  std::vector<Fp> q_plain(8ull * n), q_dedup(8ull * n);
  std::vector<uint32_t> flag_plain(n, 0), flag_dedup(n, 0);
  PipeBufs b;
  memset(&b, 0, sizeof(b));
  b.n_sets = n;
  b.msgs = msgs;
  b.sigs = sigs.data();
  b.sig_lens = lens.data();
  b.sig = sig.data();
  b.sig_status = sig_status.data();
  b.q = q_plain.data();
  b.set_flag = flag_plain.data();
  for (uint32_t t = 0; t < pre_lanes(b); ++t) stage_pre(b, t);
  b.q = q_dedup.data();
  b.set_flag = flag_dedup.data();
  b.msg_uniq = uniq.data();
  b.msg_rep = rep.data();
  b.n_uniq = u;
  for (uint32_t t = 0; t < pre_lanes(b); ++t) stage_pre(b, t);
  for (uint32_t t = 0; t < 8 * n; ++t) stage_qdup(b, t);
  for (uint32_t i = 0; i < u; ++i) uniq_out[i] = uniq[i];
  for (uint32_t i = 0; i < n; ++i) rep_out[i] = rep[i];
  memcpy(q_out, q_dedup.data(), sizeof(Fp) * 8ull * n);
  if (memcmp(q_plain.data(), q_dedup.data(), sizeof(Fp) * 8ull * n) != 0) return -1;
  if (flag_plain != flag_dedup) return -1;
  return (int)u;
}

}  // extern "C"

// ---- bls/lazy28.hpp: the 14 x 28-bit lazy representation (R' = 2^392) --------------
extern "C" {

// the raw product on digit vectors (little-endian uint32 x 14 each): out = x y / 2^392
// mod p, normalised digits
void hs_lz_mul_raw(const int32_t* x, const int32_t* y, int32_t* out, int sqr) {
  if (sqr) lz_sqr_core(x, out);
  else lz_mul_core(x, y, out);
}

// canonical Fp (48 B big-endian, plain values) through the lazy forms and back, in
// the order test_hostsim.py::test_lazy28_fp_ops expects (9 outputs of 48 B)
void hs_lz_fp_ops(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  const auto x = lz_from_fp(rd_fp(a)), y = lz_from_fp(rd_fp(b));
  const auto xy = lz_mul(x, y);
  wr_fp(lz_to_fp(xy), out);                                       // a b
  wr_fp(lz_to_fp(lz_sqr(x)), out + 48);                           // a^2
  wr_fp(lz_to_fp(lz_add(x, y)), out + 96);                        // a + b
  wr_fp(lz_to_fp(lz_sub(x, y)), out + 144);                       // a - b
  wr_fp(lz_to_fp(lz_neg(xy)), out + 192);                         // -(a b)
  wr_fp(lz_to_fp(lz_half(xy)), out + 240);                        // a b / 2
  wr_fp(lz_to_fp(lz_norm(lz_sub(xy, lz_dbl(xy)))), out + 288);    // -(a b)
  const auto s = lz_sub(lz_add(xy, xy), lz_mul(y, y));
  wr_fp(lz_to_fp(lz_mul(s, lz_norm(lz_sub(y, x)))), out + 336);   // (2ab - b^2)(b - a)
  wr_fp(lz_to_fp(x), out + 384);                                  // a (round trip)
  // lz_reduce of a large signed combination: 4 (2ab - 7 b^2 - 7 a) (|value| up to 128 p)
  const auto big = lz_sub(lz_sub(lz_add(xy, xy), lz_mulc<7>(lz_mul(y, y))), lz_mulc<7>(lz_mul(x, lz_one())));
  const auto red = lz_reduce(lz_add(lz_add(big, big), lz_add(big, big)));
  for (int k = 0; k < 13; ++k)
    if (red.d[k] < 0 || red.d[k] > (int32_t)LZ_M28) out[0] ^= 0xFF;  // digits normalised
  wr_fp(lz_to_fp(red), out + 432);
}

// Fp2 (96 B: c0 || c1) through l2_*: out = mul, sqr, mul_xi, conj, sub, mul_fp (6 x 96 B)
void hs_lz_fp2_ops(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  const auto x = l2_from_fp2(rd_fp2(a)), y = l2_from_fp2(rd_fp2(b));
  const auto m = l2_mul(x, y);
  wr_fp2(l2_to_fp2(m), out);
  wr_fp2(l2_to_fp2(l2_sqr(x)), out + 96);
  wr_fp2(l2_to_fp2(l2_mul_xi(m)), out + 192);
  wr_fp2(l2_to_fp2(l2_conj(m)), out + 288);
  wr_fp2(l2_to_fp2(l2_sub(m, l2_sqr(y))), out + 384);
  wr_fp2(l2_to_fp2(l2_mul_fp(m, y.c0)), out + 480);
}

}  // extern "C"

