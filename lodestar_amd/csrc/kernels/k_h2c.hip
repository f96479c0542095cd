// Standalone hash_to_G2 entry point (bls_gpu_hash_to_g2), one lane per message.
#include "../launchers.hpp"

using namespace bls;

__global__ __launch_bounds__(BLS_BLOCK) void k_hash_to_g2(const uint8_t* msgs, uint32_t n, uint8_t* out192) {
  uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  msg_words_from_bytes(msgs + 32ull * i, w);
  g2_serialize192(hash_to_g2(w), out192 + 192ull * i);
}

hipError_t launch_k_hash_to_g2(const uint8_t* msgs, uint32_t n, uint8_t* out192, hipStream_t s) {
  k_hash_to_g2<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(msgs, n, out192);
  return hipGetLastError();
}

// Signature.fromBytes(bytes, affine, validate) for n compressed signatures: the same
// decoder the verify path runs (g2_decompress96), then the exact G2 membership test.
__global__ __launch_bounds__(BLS_BLOCK) void k_g2_decompress(const uint8_t* in96, uint32_t n, int validate,
                                                             uint8_t* out192, int32_t* codes) {
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  G2A a;
  int32_t code = g2_decompress96(in96 + 96ull * i, a);
  if (code == BLS_OK && validate && !a.inf && !g2_in_subgroup(a)) code = BLS_POINT_NOT_IN_GROUP;
  if (code != BLS_OK) {
    a.inf = true;
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  g2_serialize192(a, out192 + 192ull * i);
  codes[i] = code;
}

hipError_t launch_k_g2_decompress(const uint8_t* in96, uint32_t n, int validate, uint8_t* out192, int32_t* codes,
                                  hipStream_t s) {
  k_g2_decompress<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(in96, n, validate, out192, codes);
  return hipGetLastError();
}

// Signature.aggregate(sigs.map((s) => Signature.fromBytes(s, undefined, true))) for
// n_lists lists (op pools: aggregatedAttestationPool.ts:320-327,
// syncContributionAndProofPool.ts:181-185, syncCommitteeMessagePool.ts:122-129).
// Stage 1, one lane per signature: decode + G2 membership (the validate=true of
// fromBytes), the point kept affine.
__global__ __launch_bounds__(BLS_BLOCK) void k_sig_decode(const uint8_t* in96, uint32_t n, G2A* pts, int32_t* codes) {
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  G2A a;
  int32_t code = g2_decompress96(in96 + 96ull * i, a);
  if (code == BLS_OK && !a.inf && !g2_in_subgroup(a)) code = BLS_POINT_NOT_IN_GROUP;
  pts[i] = a;
  codes[i] = code;
}

// Stage 2, one lane per list: the first decode error in list order rejects the list
// (fromBytes runs over the list before aggregate), an empty list is
// EMPTY_AGGREGATE_ARRAY; otherwise the sum, compressed.
__global__ __launch_bounds__(BLS_BLOCK) void k_sig_sum(const G2A* pts, const int32_t* sig_codes, const uint32_t* off,
                                                       uint32_t n_lists, uint8_t* out96, int32_t* codes) {
  const uint32_t l = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (l >= n_lists) return;
  const uint32_t beg = off[l], end = off[l + 1];
  int32_t code = beg == end ? BLS_EMPTY_AGGREGATE : BLS_OK;
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t i = beg; i < end && code == BLS_OK; ++i) {
    if (sig_codes[i] != BLS_OK) code = sig_codes[i];
    else if (!pts[i].inf) acc = jac_add_aff(acc, pts[i]);
  }
  codes[l] = code;
  G2A s;
  if (code == BLS_OK) {
    s = jac_to_aff(acc);
  } else {
    s.inf = true;
    s.x = fp2_zero();
    s.y = fp2_zero();
  }
  g2_compress96(s, out96 + 96ull * l);
}

hipError_t launch_k_sig_aggregate(const uint8_t* in96, uint32_t n, const uint32_t* off, uint32_t n_lists, G2A* pts,
                                  int32_t* sig_codes, uint8_t* out96, int32_t* codes, hipStream_t s) {
  if (n) k_sig_decode<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(in96, n, pts, sig_codes);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  k_sig_sum<<<bls_grid_for(n_lists), BLS_BLOCK, 0, s>>>(pts, sig_codes, off, n_lists, out96, codes);
  return hipGetLastError();
}
