// SSZ signing roots on the GPU (the step before the verify path):
// computeSigningRoot(type, obj, domain) = hash_tree_root(SigningData{hash_tree_root(obj),
// domain}) (state-transition/src/util/signingRoot.ts:7-13) for the fixed-size containers
// the signature-set producers sign (state-transition/src/signatureSets/*.ts).
//
// One lane per object.  An object's leaves are 32-byte chunks of its serialization
// (integers little-endian, zero padded) or nested container roots; every internal node
// is one 64-byte SHA-256 input = two compressions, the second over the constant padding
// block.  The work is a few dozen compressions per object -- latency-bound integer ALU
// work, no HBM pressure (<= 160 B in, 32 B out per object).
#include "../launchers.hpp"

using namespace bls;

namespace {

struct Chunk {
  uint32_t w[8];  // big-endian words, as SHA-256 consumes them
};

// `len` (<= 32) bytes at p, zero padded to a chunk
__device__ __forceinline__ Chunk load_chunk(const uint8_t* p, uint32_t len) {
  Chunk c;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t at = 4u * j + k;
      v = (v << 8) | (at < len ? (uint32_t)p[at] : 0u);
    }
    c.w[j] = v;
  }
  return c;
}

__device__ __forceinline__ Chunk zero_chunk() {
  Chunk c;
#pragma unroll
  for (int j = 0; j < 8; ++j) c.w[j] = 0;
  return c;
}

// SHA-256(a || b): the SSZ internal node
__device__ Chunk hash_pair(const Chunk& a, const Chunk& b) {
  uint32_t s[8], W[16];
  sha256_init(s);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    W[j] = a.w[j];
    W[8 + j] = b.w[j];
  }
  sha256_compress(s, W);
  W[0] = 0x80000000u;  // padding block of a 64-byte message
#pragma unroll
  for (int j = 1; j < 15; ++j) W[j] = 0;
  W[15] = 512;
  sha256_compress(s, W);
  Chunk r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.w[j] = s[j];
  return r;
}

// merkleize(leaves[0..n)) padded with zero chunks to width (a power of two, <= 8)
__device__ Chunk merkleize(Chunk* leaves, int n, int width) {
  Chunk zero = zero_chunk();
  for (int k = n; k < width; ++k) leaves[k] = zero;
  for (int w = width; w > 1; w >>= 1)
    for (int k = 0; k < w / 2; ++k) leaves[k] = hash_pair(leaves[2 * k], leaves[2 * k + 1]);
  return leaves[0];
}

// hash_tree_root of one serialized object; ok = false for an unknown kind
__device__ Chunk object_root(uint32_t kind, const uint8_t* o, bool& ok) {
  Chunk l[8];
  ok = true;
  switch (kind) {
    case BLS_SSZ_ROOT:
      return load_chunk(o, 32);
    case BLS_SSZ_UINT64:
      return load_chunk(o, 8);
    case BLS_SSZ_CHECKPOINT:
      return hash_pair(load_chunk(o, 8), load_chunk(o + 8, 32));
    case BLS_SSZ_ATTESTATION_DATA:
      // {slot, index, beacon_block_root, source: Checkpoint, target: Checkpoint}
      l[0] = load_chunk(o, 8);
      l[1] = load_chunk(o + 8, 8);
      l[2] = load_chunk(o + 16, 32);
      l[3] = hash_pair(load_chunk(o + 48, 8), load_chunk(o + 56, 32));
      l[4] = hash_pair(load_chunk(o + 88, 8), load_chunk(o + 96, 32));
      return merkleize(l, 5, 8);
    case BLS_SSZ_TWO_UINT64:
      return hash_pair(load_chunk(o, 8), load_chunk(o + 8, 8));
    case BLS_SSZ_BEACON_BLOCK_HEADER:
      // {slot, proposer_index, parent_root, state_root, body_root}
      l[0] = load_chunk(o, 8);
      l[1] = load_chunk(o + 8, 8);
      l[2] = load_chunk(o + 16, 32);
      l[3] = load_chunk(o + 48, 32);
      l[4] = load_chunk(o + 80, 32);
      return merkleize(l, 5, 8);
    case BLS_SSZ_DEPOSIT_MESSAGE:
      // {pubkey: Bytes48 (two chunks), withdrawal_credentials, amount}
      l[0] = hash_pair(load_chunk(o, 32), load_chunk(o + 32, 16));
      l[1] = load_chunk(o + 48, 32);
      l[2] = load_chunk(o + 80, 8);
      return merkleize(l, 3, 4);
    case BLS_SSZ_FORK_DATA:
      return hash_pair(load_chunk(o, 4), load_chunk(o + 4, 32));
    case BLS_SSZ_SIGNING_DATA:
      return hash_pair(load_chunk(o, 32), load_chunk(o + 32, 32));
    default:
      ok = false;
      return zero_chunk();
  }
}

}  // namespace

__global__ __launch_bounds__(BLS_BLOCK) void k_ssz_roots(uint32_t kind, const uint8_t* objs, uint32_t n,
                                                         const uint8_t* domains, uint32_t domain_stride,
                                                         uint8_t* out32) {
  const uint32_t i = blockIdx.x * BLS_BLOCK + threadIdx.x;
  if (i >= n) return;
  bool ok;
  Chunk r = object_root(kind, objs + (size_t)BLS_SSZ_SIZE(kind) * i, ok);
  if (domains) r = hash_pair(r, load_chunk(domains + (size_t)domain_stride * i, 32));
  uint8_t* d = out32 + 32ull * i;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    d[4 * j] = (uint8_t)(r.w[j] >> 24);
    d[4 * j + 1] = (uint8_t)(r.w[j] >> 16);
    d[4 * j + 2] = (uint8_t)(r.w[j] >> 8);
    d[4 * j + 3] = (uint8_t)r.w[j];
  }
}

bool ssz_kind_known(uint32_t kind) {
  switch (kind) {
    case BLS_SSZ_ROOT:
    case BLS_SSZ_UINT64:
    case BLS_SSZ_CHECKPOINT:
    case BLS_SSZ_ATTESTATION_DATA:
    case BLS_SSZ_TWO_UINT64:
    case BLS_SSZ_BEACON_BLOCK_HEADER:
    case BLS_SSZ_DEPOSIT_MESSAGE:
    case BLS_SSZ_FORK_DATA:
    case BLS_SSZ_SIGNING_DATA:
      return true;
    default:
      return false;
  }
}

hipError_t launch_k_ssz_roots(uint32_t kind, const uint8_t* objs, uint32_t n, const uint8_t* domains,
                              uint32_t domain_stride, uint8_t* out32, hipStream_t s) {
  k_ssz_roots<<<bls_grid_for(n), BLS_BLOCK, 0, s>>>(kind, objs, n, domains, domain_stride, out32);
  return hipGetLastError();
}
