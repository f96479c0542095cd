"""ctypes view of the C-ABI in include/lodestar_bls.h.

The product path loads lodestar_amd/_native/liblodestar_bls.so (built in-tree by
lodestar_amd/build.py) and fails loudly if it is missing: there is no CPU
fallback anywhere in the package.
"""
from __future__ import annotations

import ctypes
from pathlib import Path

import os

# $LODESTAR_BLS_LIB: another build of the same library (A/B measurements, e.g. the
# 32-bit-digit product variant from `python -m lodestar_amd.build --variant mul32`)
LIB_PATH = Path(os.environ.get("LODESTAR_BLS_LIB") or Path(__file__).resolve().parent / "_native" / "liblodestar_bls.so")

# verdict / error codes (include/lodestar_bls.h)
CODE_OK = 0
CODE_BAD_ENCODING = 1
CODE_POINT_NOT_ON_CURVE = 2
CODE_POINT_NOT_IN_GROUP = 3
CODE_PK_IS_INFINITY = 6
CODE_INVALID_SIZE = 8
CODE_ZERO_SIGNATURE = 9
CODE_EMPTY_SET = 10
CODE_EMPTY_AGGREGATE = 11

# Error messages carry the BLST_* code the reference surfaces through @chainsafe/blst
# (only "BLST_INVALID_SIZE" is pinned by the reference's own tests, multithread.test.ts:100).
ERROR_MESSAGES = {
    CODE_BAD_ENCODING: "BLST_ERROR: BLST_BAD_ENCODING",
    CODE_POINT_NOT_ON_CURVE: "BLST_ERROR: BLST_POINT_NOT_ON_CURVE",
    CODE_POINT_NOT_IN_GROUP: "BLST_ERROR: BLST_POINT_NOT_IN_GROUP",
    CODE_PK_IS_INFINITY: "BLST_ERROR: BLST_PK_IS_INFINITY",
    CODE_INVALID_SIZE: "BLST_ERROR: BLST_INVALID_SIZE",
    CODE_ZERO_SIGNATURE: "ZERO_SIGNATURE",
    CODE_EMPTY_SET: "Empty signature set",
    CODE_EMPTY_AGGREGATE: "EMPTY_AGGREGATE_ARRAY",
}

SYMBOLS = (
    "bls_gpu_device_count",
    "bls_gpu_init",
    "bls_gpu_init_priority",
    "bls_gpu_close",
    "bls_gpu_last_error",
    "bls_gpu_load_pubkeys",
    "bls_gpu_verify",
    "bls_gpu_verify_many",
    "bls_gpu_aggregate_pubkeys",
    "bls_gpu_validate_pubkeys",
    "bls_gpu_partial",
    "bls_gpu_final_check",
    "bls_gpu_hash_to_g2",
    "bls_gpu_ssz_roots",
    "bls_gpu_g2_decompress",
    "bls_gpu_aggregate_signatures",
    "bls_gpu_sk_to_pk",
    "bls_gpu_sign",
    "bls_gpu_mad_peak",
    "bls_gpu_fp_mul_test",
    "bls_gpu_fpm_bench",
    "bls_gpu_coop_probe",
    "bls_gpu_kernel_probe",
    "bls_gpu_set_debug_flags",
    "bls_gpu_init_error",
    "bls_scratch_plan",
    "bls_gpu_admission",
    "bls_scratch_worst_kernel",
    "bls_gpu_set_scratch_budget",
    "bls_gpu_request_hw_queues",
)
ERR_ADMISSION = -4  # BLS_ERR_ADMISSION: the context would push the runtime's scratch past the budget
# SSZ kinds of bls_gpu_ssz_roots (low 8 bits: serialized size)
SSZ_ROOT = 0x000 | 32
SSZ_UINT64 = 0x100 | 8
SSZ_CHECKPOINT = 0x200 | 40
SSZ_ATTESTATION_DATA = 0x300 | 128
SSZ_TWO_UINT64 = 0x400 | 16
SSZ_BEACON_BLOCK_HEADER = 0x500 | 112
SSZ_DEPOSIT_MESSAGE = 0x600 | 88
SSZ_FORK_DATA = 0x700 | 36
SSZ_SIGNING_DATA = 0x800 | 64
DEBUG_FORCE_EXACT = 1
DEBUG_NO_MSG_DEDUP = 2
DEBUG_NO_MERGED_CHECK = 4
DEBUG_SIGAGG_ON = 8
DEBUG_SIGAGG_OFF = 16
DEBUG_NO_UNITS = 32
DEBUG_MSM = 64
DEBUG_GROUP_TEST = 128
DEBUG_MERGED_EVERY_PASS = 0x8000  # (bits 8-9 are BLS_DEBUG_PACK, 12-14 BLS_DEBUG_MLF_PL)


def DEBUG_MLF_PL(n: int) -> int:
    """items per lane of the Miller loops' f side (BLS_DEBUG_MLF_PL in lodestar_bls.h)"""
    return n << 12


def DEBUG_PACK(n: int) -> int:
    """sets per wavefront of the per-set kernel (BLS_DEBUG_PACK in lodestar_bls.h)"""
    return n << 8


class BlsBatch(ctypes.Structure):
    _fields_ = [
        ("n_sets", ctypes.c_uint32),
        ("n_reqs", ctypes.c_uint32),
        ("req_set_offsets", ctypes.c_void_p),
        ("req_batchable", ctypes.c_void_p),
        ("pubkeys", ctypes.c_void_p),
        ("set_pk_offsets", ctypes.c_void_p),
        ("pk_indices", ctypes.c_void_p),
        ("messages", ctypes.c_void_p),
        ("signatures", ctypes.c_void_p),
        ("signature_lens", ctypes.c_void_p),
        ("seed", ctypes.c_void_p),
    ]


class BlsAdmission(ctypes.Structure):
    _fields_ = [
        ("contexts_normal", ctypes.c_uint32),
        ("contexts_high", ctypes.c_uint32),
        ("hw_queues", ctypes.c_uint32),
        ("queues_in_use", ctypes.c_uint32),
        ("scratch_per_queue", ctypes.c_uint64),
        ("scratch_reserved", ctypes.c_uint64),
        ("scratch_budget", ctypes.c_uint64),
        ("hw_queues_known", ctypes.c_uint32),
    ]


class BlsStats(ctypes.Structure):
    _fields_ = [
        ("batch_retries", ctypes.c_uint32),
        ("batch_sigs_success", ctypes.c_uint32),
        ("n_chunks", ctypes.c_uint32),
        ("n_individual", ctypes.c_uint32),
        ("n_flagged", ctypes.c_uint32),
        ("device_ms", ctypes.c_double),
        ("stage_ms", ctypes.c_double * 8),
        ("n_unique_msgs", ctypes.c_uint32),
        ("merged_check", ctypes.c_uint32),
        ("n_ml_units", ctypes.c_uint32),
        ("pass_shape", ctypes.c_uint32),
    ]


def bind(lib: ctypes.CDLL) -> ctypes.CDLL:
    """Attach argtypes/restype to the entry points (also used for the CPU test harness)."""
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    if hasattr(lib, "bls_gpu_init"):
        lib.bls_gpu_device_count.restype = i32
        lib.bls_gpu_init.argtypes = [i32, ctypes.POINTER(vp)]
        lib.bls_gpu_init.restype = i32
        lib.bls_gpu_init_priority.argtypes = [i32, i32, ctypes.POINTER(vp)]
        lib.bls_gpu_init_priority.restype = i32
        lib.bls_gpu_close.argtypes = [vp]
        lib.bls_gpu_close.restype = None
        lib.bls_gpu_last_error.argtypes = [vp]
        lib.bls_gpu_last_error.restype = ctypes.c_char_p
        lib.bls_gpu_load_pubkeys.argtypes = [vp, vp, u32, u32, vp]
        lib.bls_gpu_load_pubkeys.restype = ctypes.c_int64
        lib.bls_gpu_verify.argtypes = [vp, ctypes.POINTER(BlsBatch), vp, ctypes.POINTER(BlsStats)]
        lib.bls_gpu_verify.restype = i32
        lib.bls_gpu_verify_many.argtypes = [vp, ctypes.POINTER(BlsBatch), u32, vp, ctypes.POINTER(BlsStats)]
        lib.bls_gpu_verify_many.restype = i32
        lib.bls_gpu_validate_pubkeys.argtypes = [vp, vp, u32, u32, vp]
        lib.bls_gpu_validate_pubkeys.restype = i32
        lib.bls_gpu_partial.argtypes = [vp, ctypes.POINTER(BlsBatch), u32, vp, vp, vp, ctypes.POINTER(BlsStats)]
        lib.bls_gpu_partial.restype = i32
        lib.bls_gpu_final_check.argtypes = [vp, vp, u32, vp]
        lib.bls_gpu_final_check.restype = i32
        lib.bls_gpu_aggregate_pubkeys.argtypes = [vp, vp, vp, u32, vp, vp]
        lib.bls_gpu_aggregate_pubkeys.restype = i32
        lib.bls_gpu_g2_decompress.argtypes = [vp, vp, u32, i32, vp, vp]
        lib.bls_gpu_g2_decompress.restype = i32
        lib.bls_gpu_aggregate_signatures.argtypes = [vp, vp, vp, u32, vp, vp]
        lib.bls_gpu_aggregate_signatures.restype = i32
        lib.bls_gpu_hash_to_g2.argtypes = [vp, vp, u32, vp]
        lib.bls_gpu_hash_to_g2.restype = i32
        lib.bls_gpu_ssz_roots.argtypes = [vp, u32, vp, u32, vp, u32, vp]
        lib.bls_gpu_ssz_roots.restype = i32
        lib.bls_gpu_sk_to_pk.argtypes = [vp, vp, u32, vp]
        lib.bls_gpu_sk_to_pk.restype = i32
        lib.bls_gpu_sign.argtypes = [vp, vp, vp, u32, vp]
        lib.bls_gpu_sign.restype = i32
        lib.bls_gpu_mad_peak.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        lib.bls_gpu_mad_peak.restype = i32
        lib.bls_gpu_fp_mul_test.argtypes = [vp, vp, vp, u32, vp]
        lib.bls_gpu_fp_mul_test.restype = i32
        dp = ctypes.POINTER(ctypes.c_double)
        lib.bls_gpu_fpm_bench.argtypes = [vp, u32, u32, dp, dp]
        lib.bls_gpu_fpm_bench.restype = i32
        lib.bls_gpu_coop_probe.argtypes = [vp, ctypes.c_char_p, u32, u32, dp, dp, vp]
        lib.bls_gpu_coop_probe.restype = i32
        lib.bls_gpu_kernel_probe.argtypes = [vp, ctypes.c_char_p, u32, u32, dp]
        lib.bls_gpu_kernel_probe.restype = i32
        lib.bls_gpu_set_debug_flags.argtypes = [vp, u32]
        lib.bls_gpu_set_debug_flags.restype = i32
        lib.bls_gpu_init_error.argtypes = []
        lib.bls_gpu_init_error.restype = ctypes.c_char_p
        lib.bls_scratch_plan.argtypes = [u32, u32, u32, ctypes.POINTER(BlsAdmission)]
        lib.bls_scratch_plan.restype = i32
        lib.bls_gpu_admission.argtypes = [i32, ctypes.POINTER(BlsAdmission)]
        lib.bls_gpu_admission.restype = i32
        lib.bls_scratch_worst_kernel.argtypes = []
        lib.bls_scratch_worst_kernel.restype = ctypes.c_char_p
        lib.bls_gpu_set_scratch_budget.argtypes = [ctypes.c_uint64]
        lib.bls_gpu_set_scratch_budget.restype = None
        lib.bls_gpu_request_hw_queues.argtypes = [u32]
        lib.bls_gpu_request_hw_queues.restype = i32
    return lib


_LIB: ctypes.CDLL | None = None
DEFAULT_HW_QUEUES = 24
HW_QUEUES_REQUEST: int | None = None  # bls_gpu_request_hw_queues' code at load (None: not asked)


def load_library() -> ctypes.CDLL:
    """Load the in-tree HIP library; raises (never falls back) when it is absent."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -m lodestar_amd.build` "
                "(or __graft_entry__.build()); there is no CPU fallback"
            )
        lib = bind(ctypes.CDLL(str(LIB_PATH)))
        # one hardware queue per context (the runtime reads the count once, when it
        # initialises): the host's request, made here before this process's first HIP
        # call through the library; $BLS_KEEP_HW_QUEUES=1 leaves HIP's default.  The
        # returned code says whether it applied (bls_gpu_request_hw_queues).
        global HW_QUEUES_REQUEST
        if not os.environ.get("BLS_KEEP_HW_QUEUES"):
            HW_QUEUES_REQUEST = int(lib.bls_gpu_request_hw_queues(DEFAULT_HW_QUEUES))
            if HW_QUEUES_REQUEST == 0:
                os.environ["GPU_MAX_HW_QUEUES"] = str(DEFAULT_HW_QUEUES)  # Python's view of the C environment
        _LIB = lib
    return _LIB
