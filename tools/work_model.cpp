// Algorithmic work model of the aggregated-signature verify path: Fp (Montgomery)
// products per stage, counted by running the product's own host-compiled math
// (lodestar_amd/csrc/bls/*.hpp with BLS_COUNT_OPS) through the same curve-level calls
// the kernels make, role by role (kernels/k_chain.hip, k_pre.hip, k_gsum.hip).  The
// cooperative programs (Miller loops, final exponentiation) are counted from their
// tables instead (coop_programs.json: MUL ops per program).
//
// Build + run: python tools/work_model.py (writes lodestar_amd/_native/work_model.json).
#define BLS_COUNT_OPS 1
#define BLS_LAZY_POW 1  // the device's exponentiation chains (lazy28.hpp lz_pow_const)
#include <stdio.h>

#include "bls/hash_to_curve.hpp"
#include "bls/pairing.hpp"
#include "bls/pipeline.hpp"

unsigned long long bls_fpm_counter = 0;
unsigned long long bls_lz_norm_counter = 0;

using namespace bls;

static unsigned long long tick() {
  unsigned long long c = bls_fpm_counter;
  bls_fpm_counter = 0;
  return c;
}

int main() {
  const int N = 64;  // sets (messages, scalars) averaged over
  double pre = 0, h = 0, c = 0, rs = 0, rp = 0, gadd = 0, vset = 0, ml = 0, f12m = 0, mlq = 0, mlf = 0, mlf1 = 0, mlf4 = 0, madd = 0, mu = 0,
         dbl = 0;
  uint32_t seed[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  G2J prev = jac_infinity<Fp2>();
  for (int k = 0; k < N; ++k) {
    uint32_t w[8];
    for (int j = 0; j < 8; ++j) w[j] = 0x9e3779b9u * (uint32_t)(k * 8 + j + 1);
    // a signature-like G2 point and its compressed bytes, a G1 key
    const G2A sig = hash_to_g2(w);
    uint8_t sig96[96];
    g2_compress96(sig, sig96);
    const G1J pk = aff_mul_u64(g1_generator(), 1000003ull + (uint64_t)k);
    const uint64_t r = set_scalar(seed, (uint32_t)k);
    tick();
    // k_pre: hash_to_field + two SSWU maps (one lane each), signature decode
    Fp2 u0, u1, x0, y0, x1, y1;
    hash_to_field_fp2_x2(w, u0, u1);
    map_to_curve_sswu_fast(u0, x0, y0);
    map_to_curve_sswu_fast(u1, x1, y1);
    G2A dec;
    g2_decompress96(sig96, dec);
    pre += tick();
    // k_chain role 0: H = clear_cofactor(iso(q0) + iso(q1)), affine
    const G2J P = jac_add(iso_map_jac(x0, y0), iso_map_jac(x1, y1));
    const G2J Hj = g2_clear_cofactor(P);
    const Fp ni = fp_inv_gcd(fp_add(fp_sqr(Hj.z.c0), fp_sqr(Hj.z.c1)));
    const Fp2 zi = Fp2{fp_mul(Hj.z.c0, ni), fp_neg(fp_mul(Hj.z.c1, ni))};
    const Fp2 zi2 = fp2_sqr(zi);
    (void)fp2_mul(Hj.x, zi2);
    (void)fp2_mul(Hj.y, fp2_mul(zi2, zi));
    h += tick();
    // role 1: psi(sig) == [x] sig
    (void)jac_eq(g2_psi(jac_from_aff(sig)), jac_neg(aff_mul_u64(sig, (uint64_t)BLS_X_ABS)));
    c += tick();
    // role 2: [r] sig, r = a + b mu applied as [a] sig + [b] (-psi^2 sig) (curve.hpp
    // jac_mul_glv, k_chain's g2_mul_r)
    uint32_t ga, gb;
    glv_split(r, ga, gb);
    G2J T2[15];
    const G2J RS = jac_mul_glv<Fp2>(jac_from_aff(sig), ga, gb, T2);
    rs += tick();
    // role 3: [r] pk (sigma = [mu] on G1)
    G1J T1[15];
    const G1J rpk = jac_mul_glv<Fp>(pk, ga, gb, T1);
    rp += tick();
    // k_mlq: the twist-point chain and its 68 lines evaluated at P
    {
      const G1Eval P = g1_eval_affine_from_jac(rpk);  // (the inversion is no Fp product)
      G2Proj T;
      T.x = sig.x;
      T.y = sig.y;
      T.z = fp2_one();
      Fp2 c0, c1, c2;
      for (int bit = 62; bit >= 0; --bit) {
        miller_dbl_step(T, c0, c1, c2);
        (void)fp2_mul_fp(c1, P.xz), (void)fp2_mul_fp(c2, P.y);
        if ((BLS_X_ABS >> bit) & 1ull) {
          miller_add_step(T, sig, c0, c1, c2);
          (void)fp2_mul_fp(c1, P.xz), (void)fp2_mul_fp(c2, P.y);
        }
      }
      mlq += tick();
      // k_mlf: two pairs per f -- 62 squarings and 68 paired line products (fp12_mul_line2)
      Fp12 g = fp12_one();
      for (int bit = 62; bit >= 0; --bit) {
        if (bit != 62) g = fp12_sqr(g);
        for (int rep = 0; rep < (((BLS_X_ABS >> bit) & 1ull) ? 2 : 1); ++rep)
          g = fp12_mul_line2(g, c0, c1, c2, c0, c1, c2);
      }
      mlf += tick() / 2.0;
      // k_mlf with one pair per f (few sets in flight): 62 squarings and 68 line products
      Fp12 g1 = fp12_one();
      for (int bit = 62; bit >= 0; --bit) {
        if (bit != 62) g1 = fp12_sqr(g1);
        for (int rep = 0; rep < (((BLS_X_ABS >> bit) & 1ull) ? 2 : 1); ++rep) g1 = fp12_mul_line(g1, c0, c1, c2);
      }
      mlf1 += tick();
      // four pairs per f (many sets in flight): 62 squarings and 2 x 68 paired line products
      Fp12 g4 = fp12_one();
      for (int bit = 62; bit >= 0; --bit) {
        if (bit != 62) g4 = fp12_sqr(g4);
        for (int rep = 0; rep < (((BLS_X_ABS >> bit) & 1ull) ? 4 : 2); ++rep)
          g4 = fp12_mul_line2(g4, c0, c1, c2, c0, c1, c2);
      }
      mlf4 += tick() / 4.0;
    }
    // k_mls: one SIMT Miller loop per set (f of its own, no squaring shared)
    const Fp12 f = miller_loop(g1_eval_from_jac(rpk), sig);
    ml += tick();
    (void)fp12_mul(f, f);
    f12m += tick();
    // k_gsum: one G2 addition per summed point; k_vset: one affine conversion per group
    prev = jac_add(prev, RS);
    gadd += tick();
    // k_msm: one mixed addition per (window, digit) entry, the mu image of the b-half
    // point, doublings of the window scaling
    G2J acc2 = jac_add_aff(RS, sig);
    madd += tick();
    (void)g2_mu(jac_from_aff(sig));
    mu += tick();
    acc2 = jac_dbl(acc2);
    dbl += tick();
    const Fp vi = fp_inv_gcd(fp_add(fp_sqr(RS.z.c0), fp_sqr(RS.z.c1)));
    const Fp2 vz = Fp2{fp_mul(RS.z.c0, vi), fp_neg(fp_mul(RS.z.c1, vi))};
    const Fp2 vz2 = fp2_sqr(vz);
    (void)fp2_mul(RS.x, vz2);
    (void)fp2_mul(RS.y, fp2_mul(vz2, vz));
    vset += tick();
  }
  printf("{\"sets_averaged\": %d, \"k_pre\": %.1f, \"chain_h\": %.1f, \"chain_subgroup\": %.1f, "
         "\"chain_r_sig\": %.1f, \"chain_r_pk\": %.1f, \"gsum_add\": %.1f, \"vset\": %.1f, \"ml_simt\": %.1f, "
         "\"fp12_mul\": %.1f, \"ml_lines\": %.1f, \"ml_f_pair\": %.1f, \"ml_f_one\": %.1f, \"ml_f_quad\": %.1f, \"msm_madd\": %.1f, "
         "\"msm_mu\": %.1f, \"g2_dbl\": %.1f}\n",
         N, pre / N, h / N, c / N, rs / N, rp / N, gadd / N, vset / N, ml / N, f12m / N, mlq / N, mlf / N, mlf1 / N, mlf4 / N, madd / N,
         mu / N, dbl / N);
  return 0;
}
