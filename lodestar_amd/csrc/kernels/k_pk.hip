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

// getAggregatedPubkey (chain/bls/utils.ts:5-16) as a reduction, one wavefront per
// aggregate set of >= agg_min keys (b.agg_sets): lane l sums keys l, l + 64, ... of the
// set with mixed additions (table points are affine), then six levels of a tree over the
// lanes' partial sums in LDS.  An aggregate of k keys costs ceil(k / 64) + 6 additions
// of latency instead of k - 1 (cfg3's 512-key aggregates: 14 instead of 511).  The sum
// is a group element, so the order of additions changes nothing downstream (every
// consumer works on the point: the serialized aggregate is its canonical affine form).
// Table gathers stay array-of-structures: a key is one random 100-byte read.
__global__ __launch_bounds__(BLS_BLOCK) void k_pk_agg(PipeBufs b) {
  __shared__ G1J part[BLS_BLOCK];
  const uint32_t lane = threadIdx.x;
  const uint32_t i = b.agg_sets[blockIdx.x];
  const uint32_t beg = b.set_pk_off[i], end = b.set_pk_off[i + 1];
  G1J acc = jac_infinity<Fp>();
  bool bad = false;
  for (uint32_t k = beg + lane; k < end; k += BLS_BLOCK) {
    const uint32_t idx = b.pk_idx[k];
    if (idx >= b.pk_table_n) bad = true;
    else acc = jac_add_aff(acc, b.pk_table[idx]);
  }
  part[lane] = acc;
  __syncthreads();
  for (uint32_t s = BLS_BLOCK / 2; s >= 1; s >>= 1) {
    if (lane < s) part[lane] = jac_add(part[lane], part[lane + s]);
    __syncthreads();
  }
  const bool any_bad = __any(bad);
  if (lane == 0) {
    const G1J sum = part[0];
    b.pk[i] = sum;
    b.pk_status[i] = any_bad ? BLS_BAD_ENCODING : BLS_OK;
    if (b.pk_inf) b.pk_inf[i] = (!any_bad && jac_is_inf(sum)) ? 1 : 0;
  }
}

hipError_t launch_k_pk_agg(const PipeBufs& b, hipStream_t s) {
  if (b.n_agg == 0) return hipSuccess;
  k_pk_agg<<<b.n_agg, BLS_BLOCK, 0, s>>>(b);
  return hipGetLastError();
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
  BLS_TAIL_PRIO();
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
