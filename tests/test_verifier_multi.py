"""The multi-device GpuBlsVerifier's host logic on the CPU: device
slots with their own contexts, least-loaded routing of the reference's 128-set jobs
(multithread/index.ts:153-166,199-233), the in-process split of a large non-batchable
call (a shard per slot -> Fp12 partials -> one final check, lodestar_amd/shard.py's
exchange without a process group) and its re-run as the reference's jobs when a set
does not decode.  Contexts are the token stand-ins of tests/_standin.py; the same
paths with real signatures on the GPU: tests/test_gpu_multi.py."""
from __future__ import annotations

import hashlib
from concurrent.futures import wait

import pytest

from lodestar_amd.verifier import BlsError, GpuBlsVerifier, SignatureSet, set_weight
from tests._standin import INVALID, VALID, TokenCtx, token_maybe_batch


def _sets(n, bad=(), short=()):
    out = []
    for i in range(n):
        sig = INVALID if i in bad else VALID
        if i in short:
            sig = bytes(32)
        out.append(SignatureSet(i, hashlib.sha256(b"m%d" % i).digest(), sig))
    return out


def _verifier(devices, contexts=2, delay_s=0.01, **kw):
    made = []

    def make(dev, high):
        c = TokenCtx(dev, high, delay_s)
        made.append(c)
        return c

    v = GpuBlsVerifier(devices=devices, n_contexts=contexts, context_factory=make, **kw)
    return v, made


def test_set_weight():
    assert set_weight(7) == 1.0 and set_weight(bytes(96)) == 1.0 and set_weight([3]) == 1.0
    assert set_weight(list(range(512))) == pytest.approx(1.5)


def test_contexts_per_slot_and_main_lane():
    v, made = _verifier([0, 1, 1], contexts=2)
    try:
        assert [c.device for c in made] == [0, 0, 0, 1, 1, 1, 1]  # the main lane first, on slot 0's device
        assert made[0].high and not any(c.high for c in made[1:])
        assert v._ctx_slot == [0, 0, 1, 1, 2, 2]
    finally:
        v.close()


def test_jobs_routed_to_least_loaded_slot():
    """Concurrent non-batchable calls spread over both slots; each slot runs about half
    of the set weight (the slot with less outstanding weight takes the next job)."""
    v, _ = _verifier([0, 1], contexts=2, delay_s=0.02, max_sets_per_call=128)
    try:
        futs = [v.verify_signature_sets_async(_sets(128)) for _ in range(24)]
        wait(futs, timeout=60)
        assert [f.result() for f in futs] == [True] * 24
        w = [s["weight"] for s in v.slot_stats]
        assert sum(w) == 24 * 128
        assert min(w) >= 0.3 * sum(w), v.slot_stats
        assert all(s["calls"] >= 4 for s in v.slot_stats)
    finally:
        v.close()


def test_aggregate_sets_weigh_more():
    """A slot running a call of 512-key aggregates counts 1.5 per set of outstanding weight."""
    v, _ = _verifier([0, 1], contexts=1, delay_s=0.05)
    try:
        sets = [SignatureSet(list(range(512)), hashlib.sha256(b"a%d" % i).digest(), VALID) for i in range(4)]
        assert v.verify_signature_sets(sets) is True
        assert sum(s["weight"] for s in v.slot_stats) == pytest.approx(4 * 1.5)
    finally:
        v.close()


def test_split_call_valid_and_invalid():
    """A non-batchable call of >= split_call_min_sets sets: one partial per slot (shard
    sizes differ by at most 1), one final check; a call with an invalid set is false and
    its shard is the one localised."""
    v, made = _verifier([0, 1, 2], contexts=1, split_call_min_sets=64)
    try:
        assert v.verify_signature_sets(_sets(300)) is True
        parts = sorted(n for c in made for kind, n in c.calls if kind == "partial")
        assert parts == [100, 100, 100]
        assert sum(1 for c in made for kind, _ in c.calls if kind == "final_check") == 1
        assert v.split_stats["calls"] == 1 and v.split_stats["failed"] == 0
        assert v.verify_signature_sets(_sets(300, bad={250})) is False
        assert v.split_stats["failed"] == 1 and v.split_stats["bad_shards"] == [2]
        # non-batchable calls move no worker counter (worker.ts:90-97)
        tp = v.metrics.blsThreadPool
        assert tp.batchRetries.get() == 0 and tp.batchSigsSuccess.get() == 0
        # below the threshold, or batchable: the reference's jobs
        assert v.verify_signature_sets(_sets(63)) is True
        assert v.verify_signature_sets(_sets(300), batchable=True) is True
        assert v.split_stats["calls"] == 2
    finally:
        v.close()


def test_split_call_error_rerun_as_jobs():
    """A set that does not decode: the split call re-runs as the reference's 128-set jobs,
    so the rejection is the one the reference's Promise.all gives (the job of the erroring
    set rejects; a wrong-but-decodable set elsewhere does not hide it)."""
    v, _ = _verifier([0, 1], contexts=1, split_call_min_sets=64)
    try:
        with pytest.raises(BlsError, match="BLST_INVALID_SIZE"):
            v.verify_signature_sets(_sets(300, bad={3}, short={200}))
        assert v.split_stats["rerouted"] == 1 and v.split_stats["calls"] == 0
        # the reference: chunkifyMaximizeChunkSize(300, 128) = [0, 150), [150, 300), each
        # verifySignatureSetsMaybeBatch -> job 0 false, job 1 throws -> Promise.all rejects
        sets = [(s.pubkey, s.signing_root, s.signature) for s in _sets(300, bad={3}, short={200})]
        assert token_maybe_batch(sets[:150]) is False
        with pytest.raises(Exception, match="BLST_INVALID_SIZE"):
            token_maybe_batch(sets[150:])
    finally:
        v.close()


def test_batchable_counters_match_worker_semantics():
    """Batchable per-set calls routed over two slots: verdicts per call as the worker gives
    them (a failing chunk's requests re-verified alone, worker.ts:76-87)."""
    v, _ = _verifier([0, 1], contexts=1, delay_s=0.0)
    try:
        calls = [[s] for s in _sets(40, bad={7, 31})]
        futs = [v.verify_signature_sets_async(c, batchable=True) for c in calls]
        wait(futs, timeout=60)
        assert [f.result() for f in futs] == [i not in (7, 31) for i in range(40)]
        tp = v.metrics.blsThreadPool
        # every valid request ends in success, either by its chunk or alone
        assert tp.successJobsSignatureSetsCount.get() == 40
        # the chunks holding sets 7 and 31 failed and were re-verified request by request
        assert 1 <= tp.batchRetries.get() <= 2 and tp.batchSigsSuccess.get() <= 38
    finally:
        v.close()


def test_close_rejects_pending_split_shards():
    v, _ = _verifier([0, 1], contexts=1, delay_s=0.2, split_call_min_sets=64)
    f1 = v.verify_signature_sets_async(_sets(128))
    f2 = v.verify_signature_sets_async(_sets(128))
    v.close()
    outcomes = []
    for f in (f1, f2):
        try:
            outcomes.append(f.result(timeout=30))
        except Exception as e:  # noqa: BLE001
            outcomes.append(type(e).__name__)
    assert set(outcomes) <= {True, "QueueAborted"}
