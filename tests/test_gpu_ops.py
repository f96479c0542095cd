"""SURVEY §8f rows on the GPU: G2 signature aggregation for the op pools and the light
client's isValidBlsAggregate (rank 4), and the state transition's inline
verifySignatureSet (rank 3), against the oracle and the reference's semantics."""
from __future__ import annotations

import hashlib

import pytest

from lodestar_amd._abi import CODE_EMPTY_AGGREGATE, CODE_POINT_NOT_IN_GROUP
from lodestar_amd.verifier import BlsError, SignatureSet

pytestmark = pytest.mark.gpu


def _h(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


@pytest.fixture(scope="module")
def ctx(golden):
    """Own context with the 100 interop keys (KAT-2) at table indices 0..99."""
    from lodestar_amd.native import GpuContext

    c = GpuContext(0)
    pks = b"".join(bytes.fromhex(h) for h in golden["kat2_interop_pubkeys"])
    assert (c.load_pubkeys(pks, 48) == 0).all()
    yield c
    c.close()


def _sks(oracle, n):
    return [oracle.interop_secret_key(i).to_bytes(32, "big") for i in range(n)]


def test_signature_aggregate_bit_exact(ctx, oracle, golden):
    """Signature.aggregate(fromBytes(.., validate=true)) (aggregatedAttestationPool.ts:320-327):
    the compressed sum equals the oracle's, lists of 1, 2 and 7 signatures; an
    out-of-group signature or an empty list fails the list."""
    from lodestar_amd.aggregate import aggregate_into, signature_aggregate

    m = _h(b"committee-root")
    sigs = [s.tobytes() for s in ctx.sign(b"".join(_sks(oracle, 7)), m * 7)]
    lists = [sigs[:1], sigs[:2], sigs]
    out = signature_aggregate(ctx, lists)
    for lst, o in zip(lists, out):
        acc = None
        for s in lst:
            acc = oracle.E2.add(acc, oracle.signature_from_bytes(s))
        assert o == oracle.g2_compress(acc)
    assert aggregate_into(ctx, sigs[0], sigs[1]) == out[1]
    bad = bytes.fromhex(next(c["bytes"] for c in golden["sig_decode"] if c["name"] == "not_in_group"))
    _, codes = ctx.aggregate_signatures([sigs[:2], [sigs[0], bad], [], sigs[:1]])
    assert list(codes) == [0, CODE_POINT_NOT_IN_GROUP, CODE_EMPTY_AGGREGATE, 0]
    with pytest.raises(BlsError, match="EMPTY_AGGREGATE_ARRAY"):
        signature_aggregate(ctx, [[]])
    # the aggregate of the committee verifies against the aggregate pubkey (fast aggregate)
    v, _ = ctx.verify_packed(__import__("lodestar_amd.native", fromlist=["pack_requests"]).pack_requests(
        [(False, [(list(range(7)), m, out[2])])]))
    assert v[0] == 1


def test_light_client_is_valid_bls_aggregate(ctx, oracle):
    """isValidBlsAggregate (light-client/src/validation.ts:167-190): participants' keys
    aggregated on the device, signature decoded with validation, verified."""
    from lodestar_amd.aggregate import is_valid_bls_aggregate, signature_aggregate

    root = _h(b"sync-committee-root")
    part = [3, 5, 8, 13, 21, 34, 55, 89]
    sks = _sks(oracle, 100)
    sigs = [s.tobytes() for s in ctx.sign(b"".join(sks[i] for i in part), root * len(part))]
    agg = signature_aggregate(ctx, [sigs])[0]
    assert is_valid_bls_aggregate(ctx, part, root, agg) is True
    assert is_valid_bls_aggregate(ctx, part[:-1], root, agg) is False
    assert is_valid_bls_aggregate(ctx, part, _h(b"other"), agg) is False
    with pytest.raises(BlsError, match="BLST_BAD_ENCODING"):
        is_valid_bls_aggregate(ctx, part, root, bytes(96))
    with pytest.raises(BlsError, match="EMPTY_AGGREGATE_ARRAY"):
        is_valid_bls_aggregate(ctx, [], root, agg)


def test_stf_verify_signature_set(ctx, oracle):
    """verifySignatureSet (state-transition/src/util/signatureSets.ts:24-38): single and
    aggregate sets, true / false, a signature that does not decode throws; many inline
    checks in one GPU call keep their own verdicts."""
    from lodestar_amd.aggregate import signature_aggregate
    from lodestar_amd.stf import verify_signature_set, verify_signature_sets_each

    sks = _sks(oracle, 4)
    msgs = [_h(b"stf%d" % i) for i in range(4)]
    sigs = [s.tobytes() for s in ctx.sign(b"".join(sks), b"".join(msgs))]
    single = SignatureSet(2, msgs[2], sigs[2])
    wrong = SignatureSet(1, msgs[2], sigs[2])
    m = _h(b"stf-aggregate")
    agg = signature_aggregate(ctx, [[s.tobytes() for s in ctx.sign(b"".join(sks[:3]), m * 3)]])[0]
    aggregate = SignatureSet([0, 1, 2], m, agg)
    short = SignatureSet([0, 1], m, agg)
    undecodable = SignatureSet(0, msgs[0], b"\x00" * 96)
    assert verify_signature_set(ctx, single) is True
    assert verify_signature_set(ctx, wrong) is False
    assert verify_signature_set(ctx, aggregate) is True
    assert verify_signature_set(ctx, short) is False
    with pytest.raises(BlsError, match="BLST_BAD_ENCODING"):
        verify_signature_set(ctx, undecodable)
    res = verify_signature_sets_each(ctx, [single, wrong, aggregate, undecodable, short])
    assert res[:3] == [True, False, True] and isinstance(res[3], BlsError) and res[4] is False
