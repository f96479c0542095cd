// The merged signature sum S = sum_i [r_i] sig_i over a pass's live sets as a Pippenger
// multi-scalar multiplication (bucket method), replacing k_chain role 2 ([r] sig per set,
// ~1.6k Fp products) and the k_gsum levels in the merged-check path.
//
// Scalars: the set's batch scalar is r_i = a_i + b_i mu (curve.hpp glv_split / jac_mul_glv:
// a, b the two 32-bit halves of set_scalar, mu = -x^2 with [mu]Q = -psi^2(Q) on G2), so
//   S = sum_i [a_i] sig_i + [b_i] mu(sig_i):
// 2 n affine points with 32-bit scalars, four 8-bit windows, 255 buckets per window.
//
//   k_msm_bin      one lane per set: its 8 (window, digit) entries, bucket slot by atomic
//                  count; the last workgroup to finish (ticket) turns the counts into
//                  bucket and level-0 segment offsets and zeroes them for the next pass
//   k_msm_scatter  one lane per set: point references into bucket order
//   k_msm_seg      one lane per segment of <= seg points of one bucket: mixed additions
//   k_msm_bucket   one lane per bucket: the sum of its segments
//   k_msm_window   one wavefront per window: T_w = sum_d d B_{w,d} from per-lane running
//                  sums of 4 buckets, a suffix scan and a tree over the lanes in LDS,
//                  then [2^(8w)] T_w; the last window to finish (ticket) sums the four
//                  into the pass's signature sum and writes the chunk groups' virtual
//                  sets (group 0 the sum, the others infinity: f = 1; vset_write)
// Each fused step saves a dispatch: under load a one-wave kernel waits milliseconds for
// a free slot among the other passes' long waves (profiles/r03_ab_streams.json).
// The counters and tickets live in a per-context buffer zeroed once (MsmBufs::cnt).
//
// Work per pass of n sets: ~8 n mixed additions (29 Fp products each) + n/seg * ... + a
// fixed ~4k additions for the windows -- ~300 Fp products per set against ~1.6k for the
// per-set [r] sig chains.  The per-set RS are still produced (k_chain role 2 alone) when
// the merged check fails and the chunks' own sums are needed (bls_gpu.hip ensure_rs).
#define BLS_FP_D28 1
#include "../launchers.hpp"

using namespace bls;

namespace {

constexpr uint32_t MSM_W = 4, MSM_D = 255, MSM_NB = MSM_W * MSM_D;
constexpr uint32_t ENT_NONE = 0xFFFFFFFFu;

__device__ __noinline__ void msm_madd(G2J* acc, const G2A* p) { *acc = jac_add_aff(*acc, *p); }
__device__ __noinline__ void msm_add(G2J* acc, const G2J* p) { *acc = jac_add(*acc, *p); }
__device__ __noinline__ void msm_dbl(G2J* acc) { *acc = jac_dbl(*acc); }

// point reference: set index, top bit = the mu image
__device__ G2A msm_point(const PipeBufs& b, uint32_t ref) {
  const G2A s = b.sig[ref & 0x7FFFFFFFu];
  if (!(ref >> 31)) return s;
  const G2J m = g2_mu(jac_from_aff(s));  // z stays 1: psi conjugates it
  G2A r;
  r.x = m.x;
  r.y = m.y;
  r.inf = false;
  return r;
}

}  // namespace

// last workgroup of a launch: true in every lane of the workgroup that finished last;
// the launch's writes are visible to it (device-scope release / acquire fences around a
// device-scope ticket, reset for the next launch)
__device__ bool msm_last_block(uint32_t* ticket) {
  __shared__ uint32_t last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!last) return false;
  __threadfence();
  if (threadIdx.x == 0) (void)atomicExch(ticket, 0u);
  return true;
}

__global__ __launch_bounds__(BLS_BLOCK) void k_msm_bin(PipeBufs b, MsmBufs m, uint32_t seg) {
  BLS_TAIL_PRIO();
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i < b.n_sets) {
    uint32_t* ent = m.ent + 8ull * i;
    if (!b.chain_live[i]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ent[j] = ENT_NONE;
    } else {
      uint32_t sc[2];
      glv_split(set_scalar(b.seed, b.scalar_base + i), sc[0], sc[1]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w = (uint32_t)j >> 1, d = (sc[j & 1] >> (8 * w)) & 255u;
        if (d == 0) {
          ent[j] = ENT_NONE;
          continue;
        }
        const uint32_t key = w * MSM_D + d - 1;
        ent[j] = (key << 22) | atomicAdd(&m.cnt[key], 1u);
      }
    }
  }
  if (!msm_last_block(m.ticket)) return;
  // the scan, one wavefront: lane t owns buckets [16 t, 16 t + 16); off[k] = sum_{j<k}
  // cnt[j], seg_off likewise over ceil(cnt / seg) segments per bucket
  __shared__ uint32_t a[64], c[64];
  const uint32_t t = threadIdx.x, k0 = 16u * t;
  uint32_t sa = 0, sc = 0;
  for (uint32_t k = k0; k < k0 + 16u && k < MSM_NB; ++k) {
    const uint32_t n = __hip_atomic_load(&m.cnt[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sa += n;
    sc += (n + seg - 1) / seg;
  }
  a[t] = sa;
  c[t] = sc;
  __syncthreads();
  for (uint32_t off = 1; off < 64; off <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t x = t >= off ? a[t - off] : 0u, y = t >= off ? c[t - off] : 0u;
    __syncthreads();
    a[t] += x;
    c[t] += y;
    __syncthreads();
  }
  uint32_t pa = a[t] - sa, pc = c[t] - sc;  // exclusive prefixes of this lane's buckets
  for (uint32_t k = k0; k < k0 + 16u && k < MSM_NB; ++k) {
    const uint32_t n = __hip_atomic_load(&m.cnt[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    m.off[k] = pa;
    m.seg_off[k] = pc;
    pa += n;
    pc += (n + seg - 1) / seg;
    __hip_atomic_store(&m.cnt[k], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // zero for the next pass
  }
  if (t == 63) {
    m.off[MSM_NB] = a[63];
    m.seg_off[MSM_NB] = c[63];
  }
}

__global__ __launch_bounds__(BLS_BLOCK) void k_msm_scatter(PipeBufs b, MsmBufs m) {
  BLS_TAIL_PRIO();
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= b.n_sets) return;
  const uint32_t* ent = m.ent + 8ull * i;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t e = ent[j];
    if (e == ENT_NONE) continue;
    m.sorted[m.off[e >> 22] + (e & 0x3FFFFFu)] = i | ((uint32_t)(j & 1) << 31);
  }
}

// lane s: segment s of the bucket whose [seg_off[k], seg_off[k + 1]) holds it
// two wavefronts per SIMD (256 VGPRs, 864 B/lane of scratch) rather than the one that
// 352 registers gave: cfg2 +0.6 % in five alternated pairs, the signature-sum stage
// ~0.7 ms shorter (profiles/r06_ab_msm_occ.json)
#ifndef BLS_MSM_WAVES
#define BLS_MSM_WAVES 2
#endif
__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(BLS_MSM_WAVES))) void k_msm_seg(PipeBufs b, MsmBufs m, uint32_t seg) {
  BLS_TAIL_PRIO();
  const uint32_t s = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (s >= m.seg_off[MSM_NB]) return;
  uint32_t lo = 0, hi = MSM_NB;  // largest k with seg_off[k] <= s
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (m.seg_off[mid] <= s) lo = mid;
    else hi = mid;
  }
  const uint32_t beg = m.off[lo] + (s - m.seg_off[lo]) * seg;
  const uint32_t end = min(beg + seg, m.off[lo + 1]);
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t e = beg; e < end; ++e) {
    const G2A p = msm_point(b, m.sorted[e]);
    msm_madd(&acc, &p);
  }
  m.seg_sum[s] = acc;
}

__global__ __launch_bounds__(BLS_BLOCK) void k_msm_bucket(MsmBufs m) {
  BLS_TAIL_PRIO();
  const uint32_t k = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (k >= MSM_NB) return;
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t s = m.seg_off[k]; s < m.seg_off[k + 1]; ++s) {
    const G2J p = m.seg_sum[s];
    msm_add(&acc, &p);
  }
  m.bucket[k] = acc;
}

// one wavefront per window w (a 256-lane workgroup waited for a whole free CU under
// load): T_w = sum_{d=1..255} d B_{w,d}.  Lane l owns digits d = 4 l + j (j = 0..3, B_0 = O):
//   S_l = sum_j B_{4l+j},  W_l = sum_j j B_{4l+j}  (running sums, 5 additions)
//   T_w = sum_l (4 l S_l + W_l) = sum_l ([4] U_l + W_l),  U_l = sum_{k >= l, k >= 1} S_k
// U by a suffix scan over the lanes in LDS, then one tree; lane 0 scales by 2^(8 w)
__global__ __launch_bounds__(64) void k_msm_window(PipeBufs b, MsmBufs m, uint32_t groups, uint32_t vbase) {
  BLS_TAIL_PRIO();
  __shared__ G2J L[64];
  const uint32_t w = blockIdx.x, l = threadIdx.x;
  auto bucket = [&](uint32_t d) { return d ? m.bucket[w * MSM_D + d - 1] : jac_infinity<Fp2>(); };
  G2J s = bucket(4 * l + 3);  // suffix sums within the lane: s = B3, B3 + B2, ...
  G2J wl = s;                 // W = B3 + (B3 + B2) + (B3 + B2 + B1)
  for (int j = 2; j >= 0; --j) {
    const G2J bj = bucket(4 * l + (uint32_t)j);
    msm_add(&s, &bj);
    if (j > 0) msm_add(&wl, &s);
  }
  L[l] = s;  // S_l
  __syncthreads();
  G2J u = s;
  for (uint32_t off = 1; off < 64; off <<= 1) {  // suffix scan: U_l = sum_{k >= l} S_k
    G2J y = l + off < 64 ? L[l + off] : jac_infinity<Fp2>();
    __syncthreads();
    msm_add(&u, &y);
    L[l] = u;
    __syncthreads();
  }
  if (l == 0) u = jac_infinity<Fp2>();  // sum over l >= 1 only
  msm_dbl(&u);
  msm_dbl(&u);
  msm_add(&u, &wl);
  L[l] = u;
  __syncthreads();
  for (uint32_t off = 32; off >= 1; off >>= 1) {
    if (l < off) {
      G2J y = L[l + off];
      G2J z = L[l];
      msm_add(&z, &y);
      L[l] = z;
    }
    __syncthreads();
  }
  if (l == 0) {
    G2J t = L[0];
    for (uint32_t k = 0; k < 8 * w; ++k) msm_dbl(&t);
    m.win[w] = t;
  }
  if (!msm_last_block(m.ticket + 1)) return;
  // S = sum_w [2^(8w)] T_w: the chunk group 0's virtual set; the other groups are empty
  if (l == 0) {
    G2J acc = m.win[0];
    for (uint32_t k = 1; k < MSM_W; ++k) {
      const G2J p = m.win[k];
      msm_add(&acc, &p);
    }
    vset_write(b, acc, vbase);
  }
  for (uint32_t g = 1 + l; g < groups; g += 64) vset_write(b, jac_infinity<Fp2>(), vbase + g);
}

uint32_t msm_seg_len(uint32_t n_sets) {
  // ~sqrt(entries per bucket): the per-segment mixed additions and the per-bucket
  // segment additions are about equally deep
  const uint32_t per_bucket = (8u * n_sets + MSM_NB - 1) / MSM_NB;
  uint32_t seg = 8;
  while (seg * seg < per_bucket) seg *= 2;
  return seg;
}

size_t msm_seg_cap(uint32_t n_sets) { return (8ull * n_sets) / msm_seg_len(n_sets) + MSM_NB + 1; }

hipError_t launch_k_msm(const PipeBufs& b, const MsmBufs& m, uint32_t groups, uint32_t vbase, hipStream_t s) {
  const uint32_t n = b.n_sets, seg = msm_seg_len(n);
  if (n == 0) return hipErrorInvalidValue;
  k_msm_bin<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(b, m, seg);
  k_msm_scatter<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(b, m);
  k_msm_seg<<<bls_grid_for((uint32_t)msm_seg_cap(n)), BLS_BLOCK, 0, s>>>(b, m, seg);
  k_msm_bucket<<<bls_grid_for(MSM_NB), BLS_BLOCK, 0, s>>>(m);
  k_msm_window<<<MSM_W, 64, 0, s>>>(b, m, groups, vbase);
  return hipGetLastError();
}
