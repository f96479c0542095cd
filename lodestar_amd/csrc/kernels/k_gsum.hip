// Signature side of the aggregated-signature path (after k_chain.hip):
//
//   k_gsum  segmented sums of RS_i = [r_i] sig_i, one lane per segment of at most
//           GSUM_FAN points (G2 Jacobian, complete additions).  Level 0 reads the
//           sets listed in b.gsets (group-major) from b.chain, skipping sets that are
//           not live (error status, outside G2, finished by the exact path, whose f_i
//           already holds its own signature pairing); each later level sums the
//           previous level's outputs.  Segments never straddle groups, so after the
//           last level there is one sum per group (bls_gpu.hip plan_gsum).
//   k_vset  one lane per group: the sum becomes the group's virtual set for k_mln,
//           HQ = affine(sum) (one inversion), RP = -g1, so that its f is
//           ML(-g1, sum r_i sig_i) -- the single signature Miller loop blst's
//           verifyMultipleSignatures runs per batch.  A sum at infinity gives f = 1.
#define BLS_FP_INLINE 1
#include "../launchers.hpp"

using namespace bls;

namespace {

__device__ __noinline__ void g2_add_p(G2J* acc, const G2J* p) { *acc = jac_add(*acc, *p); }

__device__ G2J chain_rs(const PipeBufs& b, uint32_t i) {
  const Fp* c = b.chain + (size_t)CHAIN_WORDS * i + CH_RS;
  G2J p;
  p.x = Fp2{c[0], c[1]};
  p.y = Fp2{c[2], c[3]};
  p.z = Fp2{c[4], c[5]};
  return p;
}

}  // namespace

__global__ __launch_bounds__(BLS_BLOCK) void k_gsum(PipeBufs b, const uint32_t* seg, uint32_t n_seg, const G2J* in,
                                                    G2J* out) {
  BLS_TAIL_PRIO();
  const uint32_t k = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (k >= n_seg) return;
  const uint32_t beg = seg[2 * k], end = seg[2 * k + 1];
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t j = beg; j < end; ++j) {
    G2J p;
    if (in) {
      p = in[j];
    } else {
      const uint32_t i = b.gsets[j];
      if (!b.chain_live[i]) continue;
      p = chain_rs(b, i);
    }
    g2_add_p(&acc, &p);
  }
  out[k] = acc;
}

__global__ __launch_bounds__(BLS_BLOCK) void k_vset(PipeBufs b, const G2J* sums, uint32_t n_groups, uint32_t vbase) {
  BLS_TAIL_PRIO();
  const uint32_t g = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (g >= n_groups) return;
  vset_write(b, sums[g], vbase + g);
}

// Miller-loop units: segmented sums of RP_i = [r_i] pk_i (G1 Jacobian) over each unit's
// live sets, the same segment plan as k_gsum; k_uset then writes the unit's chain entry
// (HQ of the root's first set, RP = the sum; no affine form needed on G1).
__device__ __noinline__ void g1_add_p(G1J* acc, const G1J* p) { *acc = jac_add(*acc, *p); }

__global__ __launch_bounds__(BLS_BLOCK) void k_gsum1(PipeBufs b, const uint32_t* seg, uint32_t n_seg, const G1J* in,
                                                     G1J* out) {
  BLS_TAIL_PRIO();
  const uint32_t k = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (k >= n_seg) return;
  const uint32_t beg = seg[2 * k], end = seg[2 * k + 1];
  G1J acc = jac_infinity<Fp>();
  for (uint32_t j = beg; j < end; ++j) {
    G1J p;
    if (in) {
      p = in[j];
    } else {
      const uint32_t i = b.gsets[j];
      if (!b.chain_live[i]) continue;
      const Fp* c = b.chain + (size_t)CHAIN_WORDS * i + CH_RP;
      p.x = c[0];
      p.y = c[1];
      p.z = c[2];
    }
    g1_add_p(&acc, &p);
  }
  out[k] = acc;
}

// unit u of the call: rep = the set whose HQ the unit pairs (its root's first set)
__global__ __launch_bounds__(BLS_BLOCK) void k_uset(PipeBufs b, const G1J* sums, const uint32_t* unit_rep) {
  BLS_TAIL_PRIO();
  const uint32_t u = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (u >= b.n_units) return;
  const uint32_t v = b.unit_base + u;
  const G1J s = sums[u];
  const uint32_t rep = unit_rep[u];
  if (jac_is_inf(s)) {  // no live set (errors, exact path) or a cancelling sum: f = 1
    b.chain_live[v] = 0u;
    Fp* d = reinterpret_cast<Fp*>(&b.f[v]);
    d[0] = c_one();
#pragma unroll
    for (int k = 1; k < 12; ++k) d[k] = fp_zero();
    return;
  }
  Fp* o = b.chain + (size_t)CHAIN_WORDS * v;
  const Fp* h = b.chain + (size_t)CHAIN_WORDS * rep + CH_HQ;
#pragma unroll
  for (int k = 0; k < 4; ++k) o[CH_HQ + k] = h[k];
  o[CH_RP + 0] = s.x;
  o[CH_RP + 1] = s.y;
  o[CH_RP + 2] = s.z;
  b.chain_live[v] = 1u;
}

hipError_t launch_k_gsum1(const PipeBufs& b, const uint32_t* seg, uint32_t n_seg, const G1J* in, G1J* out,
                          hipStream_t s) {
  if (n_seg == 0) return hipSuccess;
  k_gsum1<<<bls_grid_for(n_seg), BLS_BLOCK, 0, s>>>(b, seg, n_seg, in, out);
  return hipGetLastError();
}

hipError_t launch_k_uset(const PipeBufs& b, const G1J* sums, const uint32_t* unit_rep, hipStream_t s) {
  if (b.n_units == 0) return hipSuccess;
  k_uset<<<bls_grid_for(b.n_units), BLS_BLOCK, 0, s>>>(b, sums, unit_rep);
  return hipGetLastError();
}

hipError_t launch_k_gsum(const PipeBufs& b, const uint32_t* seg, uint32_t n_seg, const G2J* in, G2J* out,
                         hipStream_t s) {
  if (n_seg == 0) return hipSuccess;
  k_gsum<<<bls_grid_for(n_seg), BLS_BLOCK, 0, s>>>(b, seg, n_seg, in, out);
  return hipGetLastError();
}

hipError_t launch_k_vset(const PipeBufs& b, const G2J* sums, uint32_t n_groups, uint32_t vbase, hipStream_t s) {
  if (n_groups == 0) return hipSuccess;
  k_vset<<<bls_grid_for(n_groups), BLS_BLOCK, 0, s>>>(b, sums, n_groups, vbase);
  return hipGetLastError();
}
