// Pubkey stage: deserialize raw 96-byte keys or sum device-table keys (aggregate sets),
// plus the pubkey-table loader and the per-request status pass (small kernels).
#include "../launchers.hpp"

using namespace bls;

// First kernel of a verify call: also resets the call's device-side words, so the
// call needs no memset blits (which queue behind every context's copies and wait for
// CU slots under load): set_flag (the exact-path marks), flag_count, and the other
// slot of the two-slot first_bad_pk (the next call's; this call's slot was reset by
// the previous call, or at context creation).
__global__ __launch_bounds__(BLS_BLOCK) void k_pk(PipeBufs b) {
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i < b.n_sets) b.set_flag[i] = b.init_set_flag;
  if (i == 0) {
    *b.flag_count = 0u;
    if (b.first_bad_pk_next) *b.first_bad_pk_next = 0xFFFFFFFFu;
  }
  stage_pk(b, i);
}

__global__ __launch_bounds__(BLS_BLOCK) void k_aggregate(PipeBufs b, uint8_t* out96) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  stage_pk(b, i);
  if (i < b.n_sets) g1_serialize96(jac_to_aff(b.pk[i]), out96 + 96ull * i);
}

__global__ __launch_bounds__(BLS_BLOCK) void k_load_pubkeys(const uint8_t* pks, uint32_t n, uint32_t pk_len,
                                                            G1A* out, int32_t* codes) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  G1A a;
  int32_t c = pk_len == 48 ? g1_decompress48(pks + 48ull * i, a) : g1_deserialize96(pks + 96ull * i, a);
  if (c != BLS_OK) {
    a.inf = true;
    a.x = fp_zero();
    a.y = fp_zero();
  }
  out[i] = a;
  codes[i] = c;
}

// KeyValidate (blst PublicKey.fromBytes(bytes, validate=true) [ext], as the deposit
// path uses it, block/processDeposit.ts:56-65): decode, reject infinity, G1 subgroup.
__global__ __launch_bounds__(BLS_BLOCK) void k_validate_pubkeys(const uint8_t* pks, uint32_t n, uint32_t pk_len,
                                                                int32_t* codes) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  G1A a;
  int32_t c = pk_len == 48 ? g1_decompress48(pks + 48ull * i, a) : g1_deserialize96(pks + 96ull * i, a);
  if (c == BLS_OK && a.inf) c = BLS_PK_IS_INFINITY;
  if (c == BLS_OK && !g1_in_subgroup(a)) c = BLS_POINT_NOT_IN_GROUP;
  codes[i] = c;
}

hipError_t launch_k_validate_pubkeys(const uint8_t* pks, uint32_t n, uint32_t pk_len, int32_t* codes, hipStream_t s) {
  k_validate_pubkeys<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(pks, n, pk_len, codes);
  return hipGetLastError();
}

// Per-request status; also mirrors the statuses and the exact-path count into the
// context's host-mapped result area (read by the host after the stream syncs, no D2H
// copy blits).
__global__ __launch_bounds__(BLS_BLOCK) void k_status(PipeBufs b) {
  const uint32_t r = blockIdx.x * BLS_BLOCK + threadIdx.x;
  stage_req_status(b, r);
  if (b.req_status_host && r < b.n_reqs) b.req_status_host[r] = b.req_status[r];
  if (r == 0 && b.flag_count_host) *b.flag_count_host = b.n_sets ? *b.flag_count : 0u;
}

hipError_t launch_k_pk(const PipeBufs& b, hipStream_t s) {
  k_pk<<<bls_grid_for(b.n_sets), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
hipError_t launch_k_aggregate(const PipeBufs& b, uint8_t* out96, hipStream_t s) {
  k_aggregate<<<bls_grid_for(b.n_sets), BLS_BLOCK, 0, s>>>(b, out96);
  return hipGetLastError();
}
hipError_t launch_k_load_pubkeys(const uint8_t* pks, uint32_t n, uint32_t pk_len, G1A* out, int32_t* codes,
                                 hipStream_t s) {
  k_load_pubkeys<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(pks, n, pk_len, out, codes);
  return hipGetLastError();
}
hipError_t launch_k_status(const PipeBufs& b, hipStream_t s) {
  k_status<<<bls_grid_for(b.n_reqs), BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
}
