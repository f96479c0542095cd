"""CPU stand-in for a verifier context (test infrastructure only): the GpuContext calls
the multi-device GpuBlsVerifier makes, answered over VALIDITY TOKENS instead of curve
points, so the host logic -- routing to the least-loaded device slot, the split call's
shards, gather and single final check, the re-run of an erroring split call as the
reference's jobs, the worker counters -- runs on the CPU in milliseconds.

A set's signature is a token: 96 bytes whose first byte is 1 (valid) or 0 (invalid);
any other length is BLST_INVALID_SIZE when verified (multithread.test.ts:89-106).  The
worker semantics (chunks of 16 requests, per-request fallback, batchRetries /
batchSigsSuccess) come from the oracle's restatement of worker.ts:32-108
(oracle.bls_oracle.verify_many_signature_sets) with this predicate as
verifySignatureSetsMaybeBatch.  The GPU test of the same host logic with real
signatures is tests/test_gpu_multi.py.
"""
from __future__ import annotations

import threading
import time
from types import SimpleNamespace

import numpy as np

from oracle import bls_oracle as O

VALID = b"\x01" + bytes(95)
INVALID = bytes(96)


def token_maybe_batch(sets) -> bool:
    """verifySignatureSetsMaybeBatch over tokens (maybeBatch.ts:16-39: an empty set list
    throws, a signature that does not decode throws, else the batch verdict)."""
    if not sets:
        raise O.BlsError(O.E_EMPTY_SET)
    for _, _, sig in sets:
        if len(sig) != 96:
            raise O.BlsError(O.E_INVALID_SIZE)
    return all(sig[0] == 1 for _, _, sig in sets)


class TokenCtx:
    """One context: `delay_s` of "device time" per call, every call recorded."""

    def __init__(self, device: int, high_priority: bool = False, delay_s: float = 0.01):
        self.device = device
        self.high = high_priority
        self.delay_s = delay_s
        self.calls = []  # (kind, n_sets)
        self.lock = threading.Lock()
        self.closed = False

    def load_pubkeys(self, pks: bytes, width: int = 48) -> np.ndarray:
        return np.zeros(len(pks) // width, dtype=np.int32)

    def close(self) -> None:
        self.closed = True

    @staticmethod
    def _requests(pb):
        reqs = []
        for r in range(pb.n_reqs):
            sets = []
            for i in range(int(pb.req_set_offsets[r]), int(pb.req_set_offsets[r + 1])):
                n = int(pb.signature_lens[i]) if pb.signature_lens is not None else 96
                sets.append((i, pb.messages[32 * i:32 * i + 32].tobytes(), pb.signatures[96 * i:96 * i + n].tobytes()))
            reqs.append((bool(pb.req_batchable[r]), sets))
        return reqs

    def _run(self, kind, n):
        with self.lock:  # one call at a time per context, like ctx->mu
            self.calls.append((kind, n))
            time.sleep(self.delay_s)

    def verify_many(self, pbs):
        verdicts, retries, ok = [], 0, 0
        for pb in pbs:
            res, rt, good = O.verify_many_signature_sets(self._requests(pb), maybe_batch=token_maybe_batch)
            verdicts.append(np.array([(1 if v else 0) if kind == "success" else -v.code for kind, v in res],
                                     dtype=np.int32))
            retries += rt
            ok += good
        self._run("verify", sum(pb.n_sets for pb in pbs))
        return verdicts, SimpleNamespace(batch_retries=retries, batch_sigs_success=ok, device_ms=self.delay_s * 1e3,
                                         merged_check=0)

    def verify_packed(self, pb):
        v, st = self.verify_many([pb])
        return v[0], st

    def partial(self, pb, base: int):
        """bls_gpu_partial over tokens: the 576-byte "partial" holds the shard's count of
        invalid sets; the first set whose signature does not decode is the shard's
        error (class 1, shard-local index)."""
        assert pb.seed is not None and len(pb.seed) == 32
        self._run("partial", pb.n_sets)
        bad = 0
        for r in range(pb.n_reqs):
            for i in range(int(pb.req_set_offsets[r]), int(pb.req_set_offsets[r + 1])):
                n = int(pb.signature_lens[i]) if pb.signature_lens is not None else 96
                if n != 96:
                    return None, -O.E_INVALID_SIZE, (1, i), None
                bad += pb.signatures[96 * i] != 1
        part = np.zeros(576, dtype=np.uint8)
        part[:4] = np.frombuffer(np.uint32(bad).tobytes(), dtype=np.uint8)
        return part.tobytes(), 0, None, None

    def final_check(self, partials) -> bool:
        self._run("final_check", len(partials))
        return sum(int(np.frombuffer(p[:4], dtype=np.uint32)[0]) for p in partials) == 0
