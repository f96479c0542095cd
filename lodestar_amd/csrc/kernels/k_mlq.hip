// Miller loops split in two SIMT kernels (the aggregated-signature path's default):
//
//   k_mlq  one lane per item: the twist point T runs from Q = HQ through the 63
//          doubling and 5 addition steps of |x| = 0xd201000000010000 (bls/pairing.hpp
//          miller_dbl_step / miller_add_step) and writes each step's line, already
//          evaluated at P = RP made affine (l0, l2 x, l3 y: 6 Fp), to a line buffer -- 68
//          lines x 288 B per item, laid out line-major and lane-minor so a wavefront's
//          stores and loads are 256-byte rows;
//   k_mlf  one lane per TWO items of one product domain (a chunk, or a non-batchable
//          request: PipeBufs::ml_dom): f = prod over both pairs' lines with ONE
//          squaring of f per bit (blst's miller_loop_n likewise shares the
//          squarings), conjugated (x < 0); f of the first item, 1 in the second.  Items
//          of different domains, or the individually verified pass (units_paired = 0),
//          run one f per item.
//
// Against a fused one-lane loop (6,803 Fp products per pair, f + T + lines live together
// in one lane, 512 registers and spills; removed in round 4): the line side takes ~1,920
// products per pair with T, P and Q only; the f side 62 squarings (36) per two pairs
// plus 68 sparse line products (39) per pair -> ~5,700 products per pair, each kernel
// with half the live state.
#define BLS_FP_D28 1
#include <stdlib.h>

#include "../launchers.hpp"
#include "bls/pairing.hpp"

using namespace bls;

namespace {

constexpr int ML_EVENTS = 68;          // 63 doublings + 5 additions
constexpr int LINE_WORDS = 6 * 12;     // l0, l2, l3 (Fp2 each) as 32-bit words

__device__ __forceinline__ bool ml_live(const PipeBufs& b, uint32_t i, uint32_t units_paired) {
  if (!b.chain_live[i]) return false;
  return !(units_paired && b.set_unit && i < b.n_sets && b.set_unit[i] != UNIT_NONE);
}

// word w of line e of item k (stride = the launch's item count, padded to a wavefront)
__device__ __forceinline__ size_t line_at(uint32_t stride, uint32_t k, int e, int w) {
  return ((size_t)e * LINE_WORDS + w) * stride + k;
}

// P affine (g1_eval_affine_from_jac, z3 = 1): l0 is c0 itself
__device__ __forceinline__ void store_line(uint32_t* L, uint32_t stride, uint32_t k, int e, const G1Eval& P,
                                           const Fp2& c0, const Fp2& c1, const Fp2& c2) {
  const Fp2 l[3] = {c0, fp2_mul_fp(c1, P.xz), fp2_mul_fp(c2, P.y)};
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int w = 0; w < 12; ++w) {
      L[line_at(stride, k, e, 24 * j + w)] = l[j].c0.l[w];
      L[line_at(stride, k, e, 24 * j + 12 + w)] = l[j].c1.l[w];
    }
}

__device__ __forceinline__ void load_line(const uint32_t* L, uint32_t stride, uint32_t k, int e, Fp2& l0, Fp2& l2,
                                          Fp2& l3) {
  Fp2* l[3] = {&l0, &l2, &l3};
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int w = 0; w < 12; ++w) {
      l[j]->c0.l[w] = L[line_at(stride, k, e, 24 * j + w)];
      l[j]->c1.l[w] = L[line_at(stride, k, e, 24 * j + 12 + w)];
    }
}

// Inlined copies of field.hpp's fp12_sqr / fp12_mul_line (out of line there, which puts
// f on the stack at every call): here f stays in registers and only the Fp products are
// calls.
__device__ __forceinline__ Fp12 sqr12(const Fp12& a) {
  const Fp6 ab = fp6_mul(a.c0, a.c1);
  const Fp6 s = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  return Fp12{fp6_sub(fp6_sub(s, ab), fp6_mul_v(ab)), fp6_add(ab, ab)};
}

__device__ __forceinline__ Fp12 mul_line12(const Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3) {
  const Fp6 aa = fp6_mul_01(f.c0, l0, l2);
  const Fp6 bb = fp6_mul_1(f.c1, l3);
  const Fp6 c1 = fp6_sub(fp6_sub(fp6_mul_01(fp6_add(f.c0, f.c1), l0, fp2_add(l2, l3)), aa), bb);
  return Fp12{fp6_add(aa, fp6_mul_v(bb)), c1};
}

// prod over n consecutive items k0 .. k0 + n - 1 of their line products, one squaring of f
// per bit (n at run time: one copy of the line product, whatever the sharing)
__device__ __forceinline__ Fp12 ml_f(const uint32_t* L, uint32_t stride, uint32_t k0, uint32_t n) {
  Fp12 f = fp12_one();
  int e = 0;
  const uint64_t X = BLS_X_ABS;
  for (int bit = 62; bit >= 0; --bit) {
    if (bit != 62) f = sqr12(f);
    const int adds = (int)((X >> bit) & 1ull);
    for (int a = 0; a <= adds; ++a) {
      uint32_t g = 0;
      // two items' lines at once (fp12_mul_line2: 23 Fp2 products instead of 26; +4 % at
      // the plateau, profiles/r03_ab_mlq_mlf.json)
#pragma unroll 1
      for (; g + 1 < n; g += 2) {
        Fp2 l0, l2, l3, m0, m2, m3;
        load_line(L, stride, k0 + g, e, l0, l2, l3);
        load_line(L, stride, k0 + g + 1, e, m0, m2, m3);
        f = fp12_mul_line2(f, l0, l2, l3, m0, m2, m3);
      }
#pragma unroll 1
      for (; g < n; ++g) {
        Fp2 l0, l2, l3;
        load_line(L, stride, k0 + g, e, l0, l2, l3);
        f = mul_line12(f, l0, l2, l3);
      }
      ++e;
    }
  }
  return fp12_conj(f);
}


}  // namespace

template <int W>
__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(W, W))) void k_mlq(
    PipeBufs b, uint32_t first, uint32_t count, uint32_t units_paired, uint32_t* L, uint32_t stride,
    const uint32_t* items) {
  const uint32_t k = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (k >= count) return;
  const uint32_t i = items ? items[k] : first + k;
  if (!ml_live(b, i, units_paired)) return;
  const Fp* ch = b.chain + (size_t)CHAIN_WORDS * i;
  G1J rp;
  rp.x = ch[CH_RP + 0];
  rp.y = ch[CH_RP + 1];
  rp.z = ch[CH_RP + 2];
  const G1Eval P = g1_eval_affine_from_jac(rp);
  G2A q;
  q.x = Fp2{ch[CH_HQ + 0], ch[CH_HQ + 1]};
  q.y = Fp2{ch[CH_HQ + 2], ch[CH_HQ + 3]};
  q.inf = false;
  G2Proj T;
  T.x = q.x;
  T.y = q.y;
  T.z = fp2_one();
  Fp2 c0, c1, c2;
  int e = 0;
  const uint64_t X = BLS_X_ABS;
  for (int bit = 62; bit >= 0; --bit) {
    miller_dbl_step(T, c0, c1, c2);
    store_line(L, stride, k, e++, P, c0, c1, c2);
    if ((X >> bit) & 1ull) {
      miller_add_step(T, q, c0, c1, c2);
      store_line(L, stride, k, e++, P, c0, c1, c2);
    }
  }
}

template <int W>
__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(W, W))) void k_mlf(
    PipeBufs b, uint32_t first, uint32_t count, uint32_t units_paired, const uint32_t* L, uint32_t stride,
    const uint32_t* items, uint32_t per_lane) {
  // per_lane items k0 .. k0 + per_lane - 1 per lane: when all are live and of one product
  // domain they share one f (one squaring per bit for all of them), else each runs its
  // own; items (an index list, the individually verified pass) never share
  const uint32_t k0 = per_lane * (blockIdx.x * BLS_BLOCK + threadIdx.x);
  if (k0 >= count) return;
  const uint32_t n = min(per_lane, count - k0);
  const uint32_t i0 = items ? items[k0] : first + k0;
  // ml_dom covers the first-pass items [0, indiv_vbase) only: the individually verified
  // requests' signature sums after it never share (reading past it paired two requests'
  // sums into one f -- the verdict bug test_verify_many_merged_signature_sum_fails found)
  bool share = n > 1 && units_paired && b.ml_dom && !items && ml_live(b, i0, units_paired);
  for (uint32_t g = 1; share && g < n; ++g) {
    const uint32_t i = first + k0 + g;
    share = ml_live(b, i, units_paired) && i < b.indiv_vbase && b.ml_dom[i] == b.ml_dom[i0];
  }
  if (share) {
    b.f[i0] = ml_f(L, stride, k0, n);
    for (uint32_t g = 1; g < n; ++g) b.f[first + k0 + g] = fp12_one();
    return;
  }
  for (uint32_t g = 0; g < n; ++g) {
    const uint32_t i = items ? items[k0 + g] : first + k0 + g;
    if (ml_live(b, i, units_paired)) b.f[i] = ml_f(L, stride, k0 + g, 1);
  }
}

// ---------------------------------------------------------------------------
// k_mlf2: the f side with two lanes per item, for few sets in flight (a pass of 16,384
// sets runs as 544 wavefronts instead of 272, each with half of the f chain's products).  Lanes 2k and 2k + 1 hold the same f; per step each computes
// one of the squaring's two Fp6 products and one of the line's two mul_by_01 products
// (plus one of the Fp2 products of f.c1 l3, and both the third), swaps its products with
// its partner (DPP quad_perm [1,0,3,2]: one move per word), and both finish the step --
// 39 Fp products per lane per doubling step instead of 75 (field.hpp fp12_sqr_half_* /
// fp12_line_half_*).  Same f as ml_f(.., 1) (test_gpu_parity runs every shape).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pair_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ Fp pair_swap(const Fp& a) {
  Fp r;
#pragma unroll
  for (int w = 0; w < 12; ++w) r.l[w] = pair_swap(a.l[w]);
  return r;
}
__device__ __forceinline__ Fp2 pair_swap(const Fp2& a) { return Fp2{pair_swap(a.c0), pair_swap(a.c1)}; }
__device__ __forceinline__ Fp6 pair_swap(const Fp6& a) { return Fp6{pair_swap(a.c0), pair_swap(a.c1), pair_swap(a.c2)}; }

__device__ __forceinline__ Fp12 sqr12_pair(const Fp12& a, bool h) {
  const Fp6 m = fp12_sqr_half_prod(a, h);
  return fp12_sqr_half_join(m, pair_swap(m), h);
}

__device__ __forceinline__ Fp12 mul_line12_pair(const Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3, bool h) {
  const LineHalf own = fp12_line_half_prod(f, l0, l2, l3, h);
  return fp12_line_half_join(own, pair_swap(own.m), pair_swap(own.p), h);
}


template <int W>
__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(W, W))) void k_mlf2(
    PipeBufs b, uint32_t first, uint32_t count, uint32_t units_paired, const uint32_t* L, uint32_t stride,
    const uint32_t* items) {
  const uint32_t t = blockIdx.x * BLS_BLOCK + threadIdx.x;
  const uint32_t k = t >> 1;
  const bool h = (t & 1u) != 0u;
  // both lanes of a pair take the same exits: the partner of every swap is active
  if (k >= count) return;
  const uint32_t i = items ? items[k] : first + k;
  if (!ml_live(b, i, units_paired)) return;
  Fp12 f = fp12_one();
  int e = 0;
  const uint64_t X = BLS_X_ABS;
  for (int bit = 62; bit >= 0; --bit) {
    if (bit != 62) f = sqr12_pair(f, h);
    const int adds = (int)((X >> bit) & 1ull);
    for (int a = 0; a <= adds; ++a) {
      Fp2 l0, l2, l3;
      load_line(L, stride, k, e, l0, l2, l3);
      f = mul_line12_pair(f, l0, l2, l3, h);
      ++e;
    }
  }
  if (!h) b.f[i] = fp12_conj(f);
}

// line buffer words for a launch of `count` items (stride padded to a wavefront)
size_t mlq_line_words(uint32_t count) {
  const size_t stride = ((size_t)count + BLS_BLOCK - 1) / BLS_BLOCK * BLS_BLOCK;
  return stride * ML_EVENTS * LINE_WORDS;
}

hipError_t launch_k_mlqf(const PipeBufs& b, uint32_t first, uint32_t count, bool own_only, uint32_t* lines,
                         hipStream_t s, const uint32_t* items) {
  if (count == 0) return hipSuccess;
  const uint32_t stride = (count + BLS_BLOCK - 1) / BLS_BLOCK * BLS_BLOCK;
  // k_mlq / k_mlf at one wavefront per SIMD (512 registers, no spills around the products:
  // +3 % at 12 x 16 over two per SIMD, profiles/r03_ab_mlq_mlf.json)
  const uint32_t up = (own_only || items) ? 0u : 1u;
  k_mlq<1><<<bls_grid_for(count), BLS_BLOCK, 0, s>>>(b, first, count, up, lines, stride, items);
  // Items per k_mlf lane: 2 shares f's squarings between two pairs (fewer instructions:
  // the rate when the device is VALU-bound), 1 halves the f chain (the rate when few sets
  // are in flight and the pass latency sets it): 2.22M vs 2.00M sets/s with 64k sets in
  // flight, 2.76M vs 2.90M with 128k (profiles/r03_ab_mlq_mlf.json).  By default the
  // process's sets in flight (every context's verify call, bls_sets_in_flight) pick:
  // 2 above $BLS_MLF_PL2_MIN (default 98,304) sets, 4 above $BLS_MLF_PL4_MIN (200,000:
  // 3.55M vs 3.41M sets/s at 12 x 22), else 1.  $BLS_MLF_PER_LANE = 1, 2, 4 or 3 (MLF_PAIR)
  // fixes it.  (Four items sharing f per lane PAIR, the squarings and line products split
  // over the pair, lost 6-11 %: spills and ~9 % more lane work, profiles/r06_ab_mlf_pair4.json.)
  // Up to $BLS_MLF_PAIR_MAX (16,384) sets in flight: two lanes per item (k_mlf2, MLF_PAIR;
  // at two waves per SIMD, $BLS_MLF2_WAVES=1 for one): a solo pass's f side 4.7 vs 7.1 ms
  // at 8,192 sets, 5.2 vs 7.2 ms at 16,384, but 8.8 vs 7.4 ms at 32,768
  // (profiles/r04_ab_mlf_pair.json).
  const uint32_t per_lane = b.mlf_pl ? b.mlf_pl : mlf_per_lane();
  if (per_lane == MLF_PAIR) {
    static const int w2 = [] {
      const char* e = getenv("BLS_MLF2_WAVES");
      return e && atoi(e) == 1 ? 1 : 2;
    }();
    if (w2 == 2) k_mlf2<2><<<bls_grid_for(2 * count), BLS_BLOCK, 0, s>>>(b, first, count, up, lines, stride, items);
    else k_mlf2<1><<<bls_grid_for(2 * count), BLS_BLOCK, 0, s>>>(b, first, count, up, lines, stride, items);
    return hipGetLastError();
  }
  const uint32_t lanes = (count + per_lane - 1) / per_lane;
  k_mlf<1><<<bls_grid_for(lanes), BLS_BLOCK, 0, s>>>(b, first, count, up, lines, stride, items, per_lane);
  return hipGetLastError();
}

uint32_t mlf_per_lane_fixed() {
  static const uint32_t fixed = [] {
    const char* e = getenv("BLS_MLF_PER_LANE");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4 || v == (int)MLF_PAIR) ? (uint32_t)v : 0u;
  }();
  return fixed;
}

uint64_t mlf_pair_max() {
  static const uint64_t pair_max = [] {
    const char* e = getenv("BLS_MLF_PAIR_MAX");
    return e ? (uint64_t)strtoull(e, nullptr, 10) : 16384ull;
  }();
  return pair_max;
}

// Items per k_mlf lane for the launches after the first pass (a failed merged check's
// chunk signature sums, the individually verified requests' own loops and sums): their
// items never share f, so more than one per lane only lengthens the chain that the failing
// call waits on (4 per lane ran each such launch for the whole 14 ms of a plateau pass's f
// side, profiles/r05_cfg5_fallback.json).  Two lanes per item up to $BLS_MLF_PAIR_MAX
// items, else one; $BLS_MLF_PER_LANE still fixes it; $BLS_MLF_ALONE=0 returns 0 (the
// launches keep the first pass's shape, as before round 5's change).
uint32_t mlf_per_lane_alone(uint32_t count) {
  static const bool off = [] {
    const char* e = getenv("BLS_MLF_ALONE");
    return e && atoi(e) == 0;
  }();
  if (off) return 0u;
  const uint32_t fixed = mlf_per_lane_fixed();
  if (fixed) return fixed;
  return count <= mlf_pair_max() ? MLF_PAIR : 1u;
}

uint32_t mlf_per_lane() {
  const uint32_t fixed = mlf_per_lane_fixed();
  const uint64_t pair_max = mlf_pair_max();
  static const uint64_t pl2_min = [] {
    const char* e = getenv("BLS_MLF_PL2_MIN");
    return e ? (uint64_t)strtoull(e, nullptr, 10) : 98304ull;
  }();
  static const uint64_t pl4_min = [] {
    const char* e = getenv("BLS_MLF_PL4_MIN");
    return e ? (uint64_t)strtoull(e, nullptr, 10) : 200000ull;
  }();
  if (fixed) return fixed;
  const uint64_t k = bls_sets_in_flight();
  return k > pl4_min ? 4u : (k > pl2_min ? 2u : (k > pair_max ? 1u : MLF_PAIR));
}
