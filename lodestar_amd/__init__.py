"""MI355X-native BLS12-381 signature-set verifier for Lodestar's IBlsVerifier hot path.

Layout:
  csrc/           HIP kernels (gfx950) + the C-ABI (include/lodestar_bls.h)
  _abi.py         ctypes view of the C-ABI; loads the in-tree library or raises
  native.py       GpuContext: one device, its stream and device pubkey table
  verifier.py     BlsGpuVerifier: the IBlsVerifier mirror (buffering, chunking, verdicts)
"""
__all__ = ["native", "verifier"]
