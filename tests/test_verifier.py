"""GpuBlsVerifier (lodestar_amd/verifier.py), the IBlsVerifier mirror, driven like the
reference's e2e pool tests (beacon-node/test/e2e/chain/bls/multithread.test.ts) and
its chunking unit test (test/unit/chain/bls/utils.test.ts, KAT-5)."""
from __future__ import annotations

import hashlib
import time

import pytest

from lodestar_amd.verifier import BlsError, SignatureSet, chunkify_maximize_chunk_size


def test_chunkify_maximize_chunk_size_kat5():
    # utils.test.ts:6-33 (minPerChunk 3, arrays of length 1..8)
    want = [
        [[0]], [[0, 1]], [[0, 1, 2]], [[0, 1, 2, 3]], [[0, 1, 2, 3, 4]],
        [[0, 1, 2], [3, 4, 5]], [[0, 1, 2, 3], [4, 5, 6]], [[0, 1, 2, 3], [4, 5, 6, 7]],
    ]
    for i, w in enumerate(want):
        assert chunkify_maximize_chunk_size(list(range(i + 1)), 3) == w
    assert chunkify_maximize_chunk_size([], 128) == [[]]


@pytest.fixture(scope="module")
def verifier(golden):
    from lodestar_amd.verifier import GpuBlsVerifier

    pks = b"".join(bytes.fromhex(h) for h in golden["kat2_interop_pubkeys"])
    v = GpuBlsVerifier(0, n_contexts=2, pubkeys48=pks)
    yield v
    v.close()


@pytest.fixture(scope="module")
def sets3(verifier, oracle):
    sks = [oracle.interop_secret_key(i).to_bytes(32, "big") for i in range(3)]
    msgs = [hashlib.sha256(b"pool%d" % i).digest() for i in range(3)]
    sigs = verifier._main.sign(b"".join(sks), b"".join(msgs))
    return [SignatureSet(i, msgs[i], sigs[i].tobytes()) for i in range(3)]


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [dict(), dict(batchable=True), dict(verify_on_main_thread=True)])
def test_many_valid_calls(verifier, sets3, opts):
    """testManyValidSignatures: 8 calls of 3 sets, submitted back to back."""
    futs = [verifier.verify_signature_sets_async(sets3, **opts) for _ in range(8)]
    assert [f.result(timeout=60) for f in futs] == [True] * 8


@pytest.mark.gpu
def test_many_valid_calls_spaced(verifier, sets3):
    futs = []
    for _ in range(8):
        futs.append(verifier.verify_signature_sets_async(sets3, batchable=True))
        time.sleep(0.005)
    assert [f.result(timeout=60) for f in futs] == [True] * 8


@pytest.mark.gpu
def test_first_invalid_does_not_poison_batch(verifier, sets3):
    """multithread.test.ts:89-106: a 32-byte signature rejects with BLST_INVALID_SIZE;
    the 8 batched valid calls still resolve true."""
    bad = SignatureSet(sets3[0].pubkey, sets3[0].signing_root, bytes(32))
    f_bad = verifier.verify_signature_sets_async([bad], batchable=True)
    futs = [verifier.verify_signature_sets_async(sets3, batchable=True) for _ in range(8)]
    with pytest.raises(BlsError, match="BLST_INVALID_SIZE"):
        f_bad.result(timeout=60)
    assert [f.result(timeout=60) for f in futs] == [True] * 8


@pytest.mark.gpu
def test_invalid_and_empty(verifier, sets3):
    wrong = SignatureSet(sets3[1].pubkey, sets3[0].signing_root, sets3[1].signature)
    assert verifier.verify_signature_sets(sets3 + [wrong]) is False
    assert verifier.verify_signature_sets([wrong], verify_on_main_thread=True) is False
    with pytest.raises(BlsError, match="Empty signature set"):
        verifier.verify_signature_sets([])
    # aggregate set over keys 0 and 1 with key 0's signature alone -> false
    assert verifier.verify_signature_sets([SignatureSet([0, 1], sets3[0].signing_root, sets3[0].signature)]) is False


@pytest.mark.gpu
def test_large_call_split_into_jobs(verifier, oracle):
    """A call of 300 sets becomes chunkifyMaximizeChunkSize(300, 128) = 2 jobs."""
    n = 300
    sks = b"".join(oracle.interop_secret_key(i % 100).to_bytes(32, "big") for i in range(n))
    msgs = [hashlib.sha256(b"big%d" % i).digest() for i in range(n)]
    sigs = verifier._main.sign(sks, b"".join(msgs))
    sets = [SignatureSet(i % 100, msgs[i], sigs[i].tobytes()) for i in range(n)]
    tp = verifier.metrics.blsThreadPool
    started, sigs = tp.totalJobsStarted.get(), tp.totalSigSetsStarted.get()
    assert verifier.verify_signature_sets(sets, batchable=True) is True
    assert tp.totalJobsStarted.get() - started == 2
    assert tp.totalSigSetsStarted.get() - sigs == n
    sets[150] = SignatureSet(sets[150].pubkey, msgs[0], sets[150].signature)
    assert verifier.verify_signature_sets(sets) is False


@pytest.mark.gpu
def test_metrics_reference_series(verifier, sets3):
    """metrics.bls.aggregatedPubkeys counts the keys of aggregate sets (index.ts:136,
    utils.ts:18-26) on both branches; the pool series move as index.ts:317-366 moves them."""
    m = verifier.metrics
    agg0 = m.bls.aggregatedPubkeys.get()
    ok0 = m.blsThreadPool.successJobsSignatureSetsCount.get()
    agg_set = SignatureSet([0, 1], sets3[0].signing_root, sets3[0].signature)
    assert verifier.verify_signature_sets([agg_set] + sets3) is False
    assert verifier.verify_signature_sets([agg_set], verify_on_main_thread=True) is False
    assert m.bls.aggregatedPubkeys.get() - agg0 == 4
    assert m.blsThreadPool.successJobsSignatureSetsCount.get() - ok0 == 4
    assert m.blsThreadPool.mainThreadDurationInThreadPool.count() >= 1
    assert m.blsThreadPool.jobWaitTime.count() >= 1
    assert verifier.queue_length() == 0
    text = m.expose()
    assert "lodestar_bls_aggregated_pubkeys_total" in text
    assert 'lodestar_bls_thread_pool_time_seconds_sum{workerId="' in text
