"""The multi-device GpuBlsVerifier on the GPU, on the 1-GPU box as
`devices=[0, 0]`: two device slots on one GPU, each with its own contexts and pubkey
table.  Checked against the oracle:

* routing: per-set batchable calls (gossip attestations) with invalid sets spread over
  both slots; each call's verdict is the sets' validity, and the worker counters the
  verifier's metrics report equal oracle.verify_many_signature_sets replayed over the
  exact GPU calls the verifier made (validity tokens, multithread/worker.ts:32-108);
* the split call: a non-batchable call of 512 sets split over the slots (one
  bls_gpu_partial per slot, one final exponentiation), all valid -> true, one invalid
  set -> false with its shard localised, one undecodable signature -> the reference's
  rejection (the call re-run as its 128-set jobs).
"""
from __future__ import annotations

import hashlib

import pytest

from lodestar_amd.verifier import BlsError, GpuBlsVerifier, SignatureSet

pytestmark = pytest.mark.gpu

N = 512


@pytest.fixture(scope="module")
def multi(golden):
    pks = b"".join(bytes.fromhex(h) for h in golden["kat2_interop_pubkeys"])
    # calls of at most 128 sets, so the 512 gossip sets make several calls to route
    v = GpuBlsVerifier(devices=[0, 0], n_contexts=2, pubkeys48=pks, split_call_min_sets=256, record_calls=True,
                       max_sets_per_call=128)
    yield v
    v.close()


@pytest.fixture(scope="module")
def signed(multi, oracle):
    sks = b"".join(oracle.interop_secret_key(i % 100).to_bytes(32, "big") for i in range(N))
    msgs = [hashlib.sha256(b"multi%d" % i).digest() for i in range(N)]
    sigs = multi._main.sign(sks, b"".join(msgs))
    return [SignatureSet(i % 100, msgs[i], sigs[i].tobytes()) for i in range(N)]


def _tamper(s: SignatureSet) -> SignatureSet:
    """The same signature over another message: decodes, fails the pairing check."""
    return SignatureSet(s.pubkey, hashlib.sha256(b"other" + s.signing_root).digest(), s.signature)


def test_two_slots_have_contexts(multi):
    assert multi.devices == [0, 0] and multi._slot_ctxs == [2, 2] and not multi.init_errors


def test_routed_gossip_calls_match_oracle(multi, signed, oracle):
    bad = {5, 77, 300, 301, 450}
    sets = [(_tamper(s) if i in bad else s) for i, s in enumerate(signed)]
    valid = {s.signature + s.signing_root: i not in bad for i, s in enumerate(sets)}
    multi.call_log.clear()
    tp = multi.metrics.blsThreadPool
    r0, ok0 = tp.batchRetries.get(), tp.batchSigsSuccess.get()
    before = [dict(s) for s in multi.slot_stats]
    futs = [multi.verify_signature_sets_async([s], batchable=True) for s in sets]
    got = [f.result(timeout=120) for f in futs]
    assert got == [i not in bad for i in range(N)]
    # both slots ran calls
    ran = [a["sets"] - b["sets"] for a, b in zip(multi.slot_stats, before)]
    assert sum(ran) == N and min(ran) > 0, ran
    # the worker counters: the oracle's worker semantics over the very calls the GPU ran
    def maybe_batch(toks):
        if not toks:
            raise oracle.BlsError(oracle.E_EMPTY_SET)
        return all(toks)
    want_r = want_ok = 0
    for _, jobs in multi.call_log:
        reqs = [(b, [valid[sig + msg] for _, msg, sig in js]) for b, js in jobs]
        res, rt, ok = oracle.verify_many_signature_sets(reqs, maybe_batch)
        want_r += rt
        want_ok += ok
    assert tp.batchRetries.get() - r0 == want_r
    assert tp.batchSigsSuccess.get() - ok0 == want_ok
    assert want_r >= 1


def test_split_call(multi, signed):
    s0 = dict(multi.split_stats)
    assert multi.verify_signature_sets(signed) is True
    assert multi.split_stats["calls"] == s0["calls"] + 1
    sets = list(signed)
    sets[400] = _tamper(sets[400])
    assert multi.verify_signature_sets(sets) is False
    assert multi.split_stats["failed"] == s0["failed"] + 1 and multi.split_stats["bad_shards"] == [1]
    # an undecodable signature: the call re-runs as the reference's jobs and rejects
    sets = list(signed)
    sets[10] = _tamper(sets[10])
    sets[300] = SignatureSet(sets[300].pubkey, sets[300].signing_root, bytes(32))
    with pytest.raises(BlsError, match="BLST_INVALID_SIZE"):
        multi.verify_signature_sets(sets)
    assert multi.split_stats["rerouted"] == s0["rerouted"] + 1
    # a batchable call of the same size is not split: jobs over the slots
    assert multi.verify_signature_sets(signed, batchable=True) is True
    assert multi.split_stats["calls"] == s0["calls"] + 2
