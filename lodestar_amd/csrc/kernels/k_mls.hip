// Miller loops of the aggregated-signature path, one lane per item (SIMT):
//   f_i = conj(f_{|x|, HQ_i}(RP_i))          (bls/pairing.hpp miller_loop)
// for every live item of [first, first + count): a set (RP = [r] pk, HQ = H(m)), a chunk
// or request signature sum (RP = -g1, HQ = sum r_i sig_i, k_vset) or a Miller-loop unit
// (RP = sum r_i pk_i, HQ = H(root), k_uset).  The batch equation multiplies every f_i
// of a chunk (k_fprod, k_chunk_coop), so a set's f is its own factor here: the shared
// 8-pair cooperative loops (k_mlns<8>) kept one f per eight sets instead.
//
// Why SIMT: one lane per pair keeps every Fp product in one lane's registers with no
// operand gathers, op fetch or LDS round trips, and all 64 lanes of a wavefront busy.
// It executes 6,803 Fp products per pair (no squaring of f shared across pairs) against
// 4,573 for the 8-pair cooperative loop, yet ran 2x the pairs per second on the device
// (profiles/r03_probe_ml.json: 4.1M pairs/s, one wavefront per SIMD, against 2.0M for
// k_mlns<8> solo).  The loop holds f (144 VGPRs), T and the line in registers; the
// register budget is one wavefront per SIMD.
#define BLS_FP_D28 1
#include <stdlib.h>

#include "../launchers.hpp"
#include "bls/pairing.hpp"

using namespace bls;

// units_paired: the first pass (a set paired inside its Miller-loop unit has f_i = 1
// from k_chain_done and runs no loop); 0: sets of requests verified alone run their own
template <int W>
__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(W, W))) void k_mls(PipeBufs b, uint32_t first,
                                                                                                uint32_t count,
                                                                                                uint32_t units_paired) {
  const uint32_t k = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (k >= count) return;
  const uint32_t i = first + k;
  if (!b.chain_live[i]) return;
  if (units_paired && b.set_unit && i < b.n_sets && b.set_unit[i] != UNIT_NONE) return;
  const Fp* ch = b.chain + (size_t)CHAIN_WORDS * i;
  G1J rp;
  rp.x = ch[CH_RP + 0];
  rp.y = ch[CH_RP + 1];
  rp.z = ch[CH_RP + 2];
  G2A hq;
  hq.x = Fp2{ch[CH_HQ + 0], ch[CH_HQ + 1]};
  hq.y = Fp2{ch[CH_HQ + 2], ch[CH_HQ + 3]};
  hq.inf = false;
  b.f[i] = miller_loop(g1_eval_from_jac(rp), hq);
}

hipError_t launch_k_mls(const PipeBufs& b, uint32_t first, uint32_t count, bool own_only, hipStream_t s) {
  if (count == 0) return hipSuccess;
  // one wavefront per SIMD: at two (256 registers) the loop spills 4,160 B/lane, and 16
  // contexts of that exhausted the runtime's scratch (profiles/r03_scratch_out_of_resources.txt)
  k_mls<1><<<bls_grid_for(count), BLS_BLOCK, 0, s>>>(b, first, count, own_only ? 0u : 1u);
  return hipGetLastError();
}
