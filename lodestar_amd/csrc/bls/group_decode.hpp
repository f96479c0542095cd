// Decoding one failed chunk's group tests with complement inference (bls_gpu.hip
// verify_groups).  Host code, shared with the CPU test harness (tests/native/hostsim.cpp,
// tests/test_hostsim.py::test_group_decode_complement_inference).
//
// The chunk's m requests of status OK are indexed 0 .. m-1; bit group G_j holds those with
// bit j of the index set (nbits = ceil(log2 m) groups).  A test passes iff the final
// exponentiation of its requests' product is 1, and the final exponentiation is
// multiplicative over disjoint request sets, so with the whole chunk's value FE(A):
// FE(rest_j) == 1 iff FE(G_j) == FE(A).  v[j]: bit 0 = G_j passed, bit 1 = FE(G_j) ==
// FE(A).
#pragma once

#include <stdint.h>

namespace bls {

// Returns m when every request is valid (the whole passed), the index of the one invalid
// request, or -1 when the outcome needs one test per request (two or more invalid show as
// a bit whose G_j and rest_j both fail; an index past m).
inline int32_t group_decode(uint32_t m, uint32_t nbits, bool whole_pass, const int32_t* v) {
  if (whole_pass) return (int32_t)m;
  if (m == 1) return 0;
  uint32_t bad = 0;
  for (uint32_t j = 0; j < nbits; ++j) {
    const bool one = (v[j] & 1) != 0, same = (v[j] & 2) != 0;
    if (one == same) return -1;  // both pass (impossible when the whole failed) or both fail
    if (!one) bad |= 1u << j;
  }
  return bad < m ? (int32_t)bad : -1;
}

}  // namespace bls
