// Exact single-lane per-set path (pipeline.hpp stage_exact_set) for the sets the
// cooperative kernel flags: an exceptional point addition (only reachable with
// signatures outside G2 or with negligible probability), an infinity signature, or
// an SSWU input the fast map does not cover.  Unflagged lanes return at once.
#include "../launchers.hpp"

using namespace bls;

// One wavefront per SIMD: the full 512-register budget keeps its scratch within the
// per-queue budget (lodestar_amd/build.py SCRATCH_BUDGET; at two per SIMD it spilled
// 7.3 KB/lane); the kernel is rare and its lanes mostly idle, so occupancy is moot.
__global__ __launch_bounds__(BLS_BLOCK) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_exact(PipeBufs b) {
  stage_exact_set(b, blockIdx.x * BLS_BLOCK + threadIdx.x);
}

hipError_t launch_k_exact(const PipeBufs& b, hipStream_t s) {
  k_exact<<<bls_grid_for(b.n_sets), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
