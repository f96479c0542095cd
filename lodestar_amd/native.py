"""Thin Python handle over the C-ABI (include/lodestar_bls.h) for one GPU.

`GpuContext` owns one `bls_gpu_ctx` (one device, one HIP stream, the device
pubkey table).  Buffers are numpy arrays handed over as raw pointers; the
library copies them into pinned staging, so nothing is retained after a call.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from ._abi import ERR_ADMISSION, BlsAdmission, BlsBatch, BlsStats, load_library


def _ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def _u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


class NativeError(RuntimeError):
    pass


class AdmissionError(NativeError):
    """bls_gpu_init refused the context (BLS_ERR_ADMISSION): the HIP runtime's scratch for
    the process's contexts would pass the budget (include/lodestar_bls.h bls_admission)."""


def mapped_hip_runtime() -> list[str]:
    """Paths of the HIP runtime (libamdhip64) mapped into this process: /opt/rocm's when
    the library is loaded first, torch's bundled copy (same soname) when torch was
    imported before it -- the runtime the library's kernels then run under."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})
    except OSError:
        return []


class _DlInfo(ctypes.Structure):
    _fields_ = [("dli_fname", ctypes.c_char_p), ("dli_fbase", ctypes.c_void_p), ("dli_sname", ctypes.c_char_p),
                ("dli_saddr", ctypes.c_void_p)]


def library_hip_runtime() -> str | None:
    """The libamdhip64 file the library's HIP calls bind to: dlsym through the library's
    own handle searches its dependency scope, dladdr names the object that holds the
    symbol.  (/proc/self/maps may list two copies once torch is imported after the
    library: torch loads its bundled one by another name and never initialises it unless
    torch.cuda is used.)"""
    lib = load_library()
    try:
        addr = ctypes.cast(lib.hipGetDeviceCount, ctypes.c_void_p).value
    except AttributeError:
        return None
    info = _DlInfo()
    libc = ctypes.CDLL(None)
    libc.dladdr.argtypes = [ctypes.c_void_p, ctypes.POINTER(_DlInfo)]
    if not addr or libc.dladdr(ctypes.c_void_p(addr), ctypes.byref(info)) == 0 or not info.dli_fname:
        return None
    return os.path.realpath(info.dli_fname.decode())


def scratch_plan(n_normal: int, n_high: int, hw_queues: int = 0) -> tuple[bool, dict]:
    """The library's admission accounting for n_normal + n_high contexts (no device
    needed): (admissible, the bls_admission figures)."""
    a = BlsAdmission()
    rc = load_library().bls_scratch_plan(n_normal, n_high, hw_queues, ctypes.byref(a))
    return rc == 0, {f: getattr(a, f) for f, _ in BlsAdmission._fields_}


def admission(device: int = 0) -> dict:
    """The figures for the contexts open on `device` in this process."""
    a = BlsAdmission()
    load_library().bls_gpu_admission(device, ctypes.byref(a))
    return {f: getattr(a, f) for f, _ in BlsAdmission._fields_}


@dataclass
class PackedBatch:
    """SoA form of one verifyManySignatureSets call (bls_batch)."""

    req_set_offsets: np.ndarray  # uint32[n_reqs + 1]
    req_batchable: np.ndarray  # uint8[n_reqs]
    messages: np.ndarray  # uint8[n_sets * 32]
    signatures: np.ndarray  # uint8[n_sets * 96]
    pubkeys: np.ndarray | None = None  # uint8[n_sets * 96]
    set_pk_offsets: np.ndarray | None = None  # uint32[n_sets + 1]
    pk_indices: np.ndarray | None = None  # uint32[...]
    signature_lens: np.ndarray | None = None  # uint32[n_sets]
    seed: bytes | None = None
    # the bls_batch view of these arrays, built on first use (GpuContext._batch_struct):
    # a pass of 64 calls re-packed its 64 structs under the GIL at every submission
    _cstruct: object = field(default=None, repr=False, compare=False)

    @property
    def n_sets(self) -> int:
        return int(self.req_set_offsets[-1])

    @property
    def n_reqs(self) -> int:
        return len(self.req_set_offsets) - 1


def pack_requests(requests, seed: bytes | None = None) -> PackedBatch:
    """requests: list of (batchable: bool, sets) where each set is (pk, msg32, sig).

    pk is either 96 raw bytes (uncompressed affine) or a list/tuple of device
    pubkey-table indices (all sets of one batch must use the same form).  sig may
    have any length (a length other than 96 yields BLST_INVALID_SIZE)."""
    offs = [0]
    batchable = []
    msgs, sigs, lens = [], [], []
    raw_pks, idx_offs, idx = [], [0], []
    table_mode = None
    for is_b, sets in requests:
        batchable.append(1 if is_b else 0)
        for pk, msg, sig in sets:
            this_table = not isinstance(pk, (bytes, bytearray, memoryview, np.ndarray))
            if table_mode is None:
                table_mode = this_table
            if table_mode != this_table:
                raise ValueError("mixed raw / table pubkeys in one batch")
            if table_mode:
                idx.extend(int(i) for i in pk)
                idx_offs.append(len(idx))
            else:
                pkb = bytes(pk)
                if len(pkb) != 96:
                    # the worker wire format is the 96-byte uncompressed key (index.ts:126,160);
                    # the C-ABI reads exactly 96 bytes per set
                    raise ValueError(f"raw pubkeys are 96 bytes (uncompressed affine), got {len(pkb)}")
                raw_pks.append(pkb)
            if len(msg) != 32:
                raise ValueError("signing roots are 32 bytes")
            msgs.append(bytes(msg))
            sb = bytes(sig)
            lens.append(len(sb))
            sigs.append(sb[:96].ljust(96, b"\0"))
        offs.append(len(msgs))
    n = len(msgs)
    pb = PackedBatch(
        req_set_offsets=np.array(offs, dtype=np.uint32),
        req_batchable=np.array(batchable, dtype=np.uint8),
        messages=np.frombuffer(b"".join(msgs), dtype=np.uint8).copy() if n else np.zeros(1, np.uint8),
        signatures=np.frombuffer(b"".join(sigs), dtype=np.uint8).copy() if n else np.zeros(1, np.uint8),
        seed=seed,
    )
    if any(L != 96 for L in lens):
        pb.signature_lens = np.array(lens, dtype=np.uint32)
    if table_mode:
        pb.set_pk_offsets = np.array(idx_offs, dtype=np.uint32)
        pb.pk_indices = np.array(idx if idx else [0], dtype=np.uint32)
    else:
        pb.pubkeys = np.frombuffer(b"".join(raw_pks), dtype=np.uint8).copy() if n else np.zeros(96, np.uint8)
    return pb


class GpuContext:
    def __init__(self, device: int = 0, high_priority: bool = False):
        """high_priority: the context's stream outranks normal contexts' queued kernels
        (bls_gpu_init_priority; the verifyOnMainThread latency lane)."""
        self.lib = load_library()
        ndev = self.lib.bls_gpu_device_count()
        if ndev <= device:
            raise NativeError(f"no HIP device {device} (visible: {ndev}); the verifier has no CPU fallback")
        h = ctypes.c_void_p()
        rc = self.lib.bls_gpu_init_priority(device, 1 if high_priority else 0, ctypes.byref(h))
        if rc != 0:
            msg = (self.lib.bls_gpu_init_error() or b"").decode() or f"bls_gpu_init_priority({device}) failed"
            raise (AdmissionError if rc == ERR_ADMISSION else NativeError)(msg)
        self._h = h
        self.device = device

    # -- lifecycle ------------------------------------------------------------
    def close(self) -> None:
        if self._h:
            self.lib.bls_gpu_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str):
        if rc < 0:
            msg = self.lib.bls_gpu_last_error(self._h)
            raise NativeError(f"{what}: {msg.decode() if msg else rc}")

    # -- pubkey table ---------------------------------------------------------
    def load_pubkeys(self, pks: bytes | np.ndarray, pk_len: int = 48) -> np.ndarray:
        arr = _u8(pks)
        n = arr.size // pk_len
        codes = np.zeros(max(n, 1), dtype=np.int32)
        rc = self.lib.bls_gpu_load_pubkeys(self._h, _ptr(arr), n, pk_len, _ptr(codes))
        self._check(rc, "bls_gpu_load_pubkeys")
        return codes[:n]

    def validate_pubkeys(self, pks: bytes | np.ndarray, pk_len: int = 48) -> np.ndarray:
        """KeyValidate codes (0 valid, else BLST-style code) for n keys (bls_gpu_validate_pubkeys)."""
        arr = _u8(pks)
        n = arr.size // pk_len
        codes = np.zeros(max(n, 1), dtype=np.int32)
        rc = self.lib.bls_gpu_validate_pubkeys(self._h, _ptr(arr), n, pk_len, _ptr(codes))
        self._check(rc, "bls_gpu_validate_pubkeys")
        return codes[:n]

    # -- verification -------------------------------------------------------------
    @staticmethod
    def _batch_struct(pb: PackedBatch):
        # cached on the batch: the view points at the batch's arrays, so edits in place
        # are seen; a caller that replaces one of them must build a new PackedBatch
        if pb._cstruct is not None:
            return pb._cstruct
        keep = []
        b = BlsBatch()
        b.n_sets = pb.n_sets
        b.n_reqs = pb.n_reqs
        for field in ("req_set_offsets", "req_batchable", "messages", "signatures", "pubkeys", "set_pk_offsets",
                      "pk_indices", "signature_lens"):
            a = getattr(pb, field)
            if a is not None:
                a = np.ascontiguousarray(a)
                keep.append(a)
            setattr(b, field, _ptr(a))
        seed_buf = None
        if pb.seed is not None:
            seed_buf = ctypes.create_string_buffer(bytes(pb.seed), 32)
            b.seed = ctypes.cast(seed_buf, ctypes.c_void_p)
        keep.append(seed_buf)
        pb._cstruct = (b, keep)
        return b, keep

    def verify_packed(self, pb: PackedBatch) -> tuple[np.ndarray, BlsStats]:
        b, _keep = self._batch_struct(pb)
        verdicts = np.zeros(max(pb.n_reqs, 1), dtype=np.int32)
        stats = BlsStats()
        rc = self.lib.bls_gpu_verify(self._h, ctypes.byref(b), _ptr(verdicts), ctypes.byref(stats))
        self._check(rc, "bls_gpu_verify")
        return verdicts[: pb.n_reqs], stats

    def verify_many(self, pbs: list[PackedBatch]) -> tuple[list[np.ndarray], BlsStats]:
        """Several worker messages in one submission (bls_gpu_verify_many): per-message
        verdict arrays (each as verify_packed would return it) and the totals."""
        structs, keep = (BlsBatch * max(len(pbs), 1))(), []
        for k, pb in enumerate(pbs):
            b, kp = self._batch_struct(pb)
            structs[k] = b
            keep.append(kp)
        total = sum(pb.n_reqs for pb in pbs)
        verdicts = np.zeros(max(total, 1), dtype=np.int32)
        stats = BlsStats()
        rc = self.lib.bls_gpu_verify_many(self._h, structs, len(pbs), _ptr(verdicts), ctypes.byref(stats))
        self._check(rc, "bls_gpu_verify_many")
        out, off = [], 0
        for pb in pbs:
            out.append(verdicts[off: off + pb.n_reqs])
            off += pb.n_reqs
        return out, stats

    def partial(self, pb: PackedBatch, set_index_base: int):
        """Miller-loop partial of this shard of a sharded call (bls_gpu_partial):
        (576 opaque bytes or None on an error, status 0 / -code, (class, shard-local set
        index) of the error or None, stats)."""
        if pb.seed is None:
            raise ValueError("a sharded call needs the call's shared 32-byte seed")
        b, _keep = self._batch_struct(pb)
        out = np.zeros(576, dtype=np.uint8)
        status = ctypes.c_int32(0)
        err = np.zeros(2, dtype=np.uint32)
        stats = BlsStats()
        rc = self.lib.bls_gpu_partial(self._h, ctypes.byref(b), set_index_base, _ptr(out), ctypes.byref(status),
                                      _ptr(err), ctypes.byref(stats))
        self._check(rc, "bls_gpu_partial")
        if status.value == 0:
            return out.tobytes(), 0, None, stats
        return None, status.value, (int(err[0]), int(err[1])), stats

    def final_check(self, partials: list[bytes]) -> bool:
        """FE(prod partials) == 1: the one final exponentiation of a sharded call."""
        buf = _u8(b"".join(partials))
        v = ctypes.c_int32(-1)
        rc = self.lib.bls_gpu_final_check(self._h, _ptr(buf), len(partials), ctypes.byref(v))
        self._check(rc, "bls_gpu_final_check")
        return v.value == 1

    # -- standalone primitives (parity tests, fixtures) ---------------------------
    def aggregate_pubkeys(self, index_lists) -> tuple[list[bytes], np.ndarray]:
        offs = [0]
        idx = []
        for lst in index_lists:
            idx.extend(int(i) for i in lst)
            offs.append(len(idx))
        n = len(index_lists)
        o = np.array(offs, dtype=np.uint32)
        ix = np.array(idx if idx else [0], dtype=np.uint32)
        out = np.zeros(96 * max(n, 1), dtype=np.uint8)
        codes = np.zeros(max(n, 1), dtype=np.int32)
        rc = self.lib.bls_gpu_aggregate_pubkeys(self._h, _ptr(o), _ptr(ix), n, _ptr(out), _ptr(codes))
        self._check(rc, "bls_gpu_aggregate_pubkeys")
        raw = out.tobytes()
        return [raw[96 * i: 96 * i + 96] for i in range(n)], codes[:n]

    def hash_to_g2(self, msgs: bytes | np.ndarray) -> np.ndarray:
        m = _u8(msgs)
        n = m.size // 32
        out = np.zeros(192 * max(n, 1), dtype=np.uint8)
        self._check(self.lib.bls_gpu_hash_to_g2(self._h, _ptr(m), n, _ptr(out)), "bls_gpu_hash_to_g2")
        return out[: 192 * n].reshape(n, 192)

    def ssz_roots(self, kind: int, objs: bytes | np.ndarray, domains: bytes | np.ndarray | None = None) -> np.ndarray:
        """computeSigningRoot over n serialized objects of one SSZ kind (bls_gpu_ssz_roots;
        signingRoot.ts:7-13): n x 32 signing roots, or the objects' hash_tree_roots when
        domains is None.  domains: one 32-byte domain for all, or 32 bytes per object."""
        o = _u8(objs)
        size = kind & 0xFF
        if o.size % size:
            raise ValueError(f"objects are {size} bytes each, got {o.size} bytes")
        n = o.size // size
        d, stride = None, 0
        if domains is not None:
            d = _u8(domains)
            if d.size == 32:
                stride = 0
            elif d.size == 32 * n:
                stride = 32
            else:
                raise ValueError("domains: 32 bytes, or 32 bytes per object")
        out = np.zeros(32 * max(n, 1), dtype=np.uint8)
        rc = self.lib.bls_gpu_ssz_roots(self._h, kind, _ptr(o) if n else None, n, _ptr(d), stride, _ptr(out))
        self._check(rc, "bls_gpu_ssz_roots")
        return out[: 32 * n].reshape(n, 32)

    def g2_decompress(self, sigs96: bytes | np.ndarray, validate: bool = True) -> tuple[np.ndarray, np.ndarray]:
        """Signature.fromBytes(b, affine, validate) for n 96-byte signatures:
        (n x 192 uncompressed bytes, n codes) (bls_gpu_g2_decompress)."""
        s = _u8(sigs96)
        n = s.size // 96
        out = np.zeros(192 * max(n, 1), dtype=np.uint8)
        codes = np.zeros(max(n, 1), dtype=np.int32)
        self._check(self.lib.bls_gpu_g2_decompress(self._h, _ptr(s), n, 1 if validate else 0, _ptr(out), _ptr(codes)),
                    "bls_gpu_g2_decompress")
        return out[: 192 * n].reshape(n, 192), codes[:n]

    def aggregate_signatures(self, sig_lists) -> tuple[list[bytes], np.ndarray]:
        """Signature.aggregate over lists of 96-byte signatures (each decoded with
        validate=true): (compressed sums, codes) (bls_gpu_aggregate_signatures)."""
        offs, flat = [0], []
        for lst in sig_lists:
            for sig in lst:
                b = bytes(sig)
                if len(b) != 96:
                    raise ValueError("signatures are 96 bytes (compressed G2)")
                flat.append(b)
            offs.append(len(flat))
        n_lists = len(sig_lists)
        o = np.array(offs, dtype=np.uint32)
        buf = np.frombuffer(b"".join(flat), dtype=np.uint8).copy() if flat else np.zeros(96, np.uint8)
        out = np.zeros(96 * max(n_lists, 1), dtype=np.uint8)
        codes = np.zeros(max(n_lists, 1), dtype=np.int32)
        self._check(self.lib.bls_gpu_aggregate_signatures(self._h, _ptr(buf), _ptr(o), n_lists, _ptr(out),
                                                          _ptr(codes)), "bls_gpu_aggregate_signatures")
        raw = out.tobytes()
        return [raw[96 * i: 96 * i + 96] for i in range(n_lists)], codes[:n_lists]

    def sk_to_pk(self, sks: bytes | np.ndarray) -> np.ndarray:
        s = _u8(sks)
        n = s.size // 32
        out = np.zeros(48 * max(n, 1), dtype=np.uint8)
        self._check(self.lib.bls_gpu_sk_to_pk(self._h, _ptr(s), n, _ptr(out)), "bls_gpu_sk_to_pk")
        return out[: 48 * n].reshape(n, 48)

    # ORed into every set_debug_flags call (tests run a whole module once per path)
    base_debug_flags = 0

    def set_debug_flags(self, flags: int) -> None:
        self._check(self.lib.bls_gpu_set_debug_flags(self._h, flags | self.base_debug_flags),
                    "bls_gpu_set_debug_flags")

    def mad_peak(self) -> tuple[float, float]:
        """Measured v_mad_u64_u32 rate (MAD/s) and the probe's duration (ms)."""
        rate, ms = ctypes.c_double(), ctypes.c_double()
        self._check(self.lib.bls_gpu_mad_peak(self._h, ctypes.byref(rate), ctypes.byref(ms)), "bls_gpu_mad_peak")
        return rate.value, ms.value

    def fp_mul_test(self, a: bytes, b: bytes) -> bytes:
        n = len(a) // 48
        out = ctypes.create_string_buffer(48 * max(n, 1))
        self._check(self.lib.bls_gpu_fp_mul_test(self._h, a, b, n, out), "bls_gpu_fp_mul_test")
        return out.raw[: 48 * n]

    def fpm_bench(self, lanes: int, iters: int) -> tuple[float, float]:
        ns, rate = ctypes.c_double(), ctypes.c_double()
        self._check(self.lib.bls_gpu_fpm_bench(self._h, lanes, iters, ctypes.byref(ns), ctypes.byref(rate)),
                    "bls_gpu_fpm_bench")
        return ns.value, rate.value

    def kernel_probe(self, name: str, lanes: int, reps: int) -> float:
        """Wall ms of `reps` launches of the design probe `name` over `lanes` lanes
        (kernels/k_probe.hip)."""
        ms = ctypes.c_double()
        self._check(self.lib.bls_gpu_kernel_probe(self._h, name.encode(), lanes, reps, ctypes.byref(ms)),
                    "bls_gpu_kernel_probe")
        return ms.value

    def coop_probe(self, name: str, blocks: int, reps: int, n_stamps: int = 0):
        """(us per step, ms total[, per-step s_memtime stamps of one run])"""
        us, ms = ctypes.c_double(), ctypes.c_double()
        stamps = np.zeros(n_stamps, dtype=np.uint64) if n_stamps else None
        self._check(self.lib.bls_gpu_coop_probe(self._h, name.encode(), blocks, reps, ctypes.byref(us),
                                                ctypes.byref(ms), _ptr(stamps)), "bls_gpu_coop_probe")
        if stamps is not None:
            return us.value, ms.value, stamps
        return us.value, ms.value

    def sign(self, sks: bytes | np.ndarray, msgs: bytes | np.ndarray) -> np.ndarray:
        s, m = _u8(sks), _u8(msgs)
        n = s.size // 32
        out = np.zeros(96 * max(n, 1), dtype=np.uint8)
        self._check(self.lib.bls_gpu_sign(self._h, _ptr(s), _ptr(m), n, _ptr(out)), "bls_gpu_sign")
        return out[: 96 * n].reshape(n, 96)
