// Exact single-lane per-set path (pipeline.hpp stage_exact_set) for the sets the
// cooperative kernel flags: an exceptional point addition (only reachable with
// signatures outside G2 or with negligible probability), an infinity signature, or
// an SSWU input the fast map does not cover.  Unflagged lanes return at once.
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK, 2) void k_exact(PipeBufs b) {
  stage_exact_set(b, blockIdx.x * BLS_BLOCK + threadIdx.x);
}

hipError_t launch_k_exact(const PipeBufs& b, hipStream_t s) {
  k_exact<<<bls_grid_for(b.n_sets), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
