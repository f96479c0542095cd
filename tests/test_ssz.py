"""SSZ signing roots (signingRoot.ts:7-13, domain.ts:9-45).

CPU: the oracle (oracle/ssz_oracle.py) against the reference's own data -- the mainnet
block chain of beacon-node/test/unit/sync/backfill/blocks.json (hash_tree_root(block i) ==
block i+1's parent_root) and the KAT-1 deposit signing root -- and the committed vectors.
GPU: k_ssz_roots through the C-ABI against the same fixtures, bit-exact.
"""
from __future__ import annotations

import json
from pathlib import Path

import pytest

from oracle import ssz_oracle as S

G = json.loads((Path(__file__).resolve().parent / "golden" / "ssz_golden.json").read_text())


def test_oracle_reproduces_mainnet_block_roots():
    for blk, want in zip(G["blocks"], G["expected_roots"]):
        assert S.block_json_root_phase0(blk).hex() == want


def test_oracle_kat1_deposit_signing_root():
    k = G["kat1_deposit"]
    dom = S.compute_domain(bytes.fromhex("03000000"), bytes.fromhex(k["fork_version"]),
                           bytes.fromhex(k["genesis_validators_root"]))
    assert dom.hex() == k["domain"]
    obj = S.deposit_message_root(bytes.fromhex(k["pubkey"]), bytes.fromhex(k["withdrawal_credentials"]), k["amount"])
    assert S.compute_signing_root(obj, dom).hex() == k["signing_root"]


def test_oracle_vectors():
    for kind, v in G["vectors"].items():
        for o, d, r, sr in zip(v["objs"], v["domains"], v["roots"], v["signing_roots"]):
            root = S.root_of_serialized(kind, bytes.fromhex(o))
            assert root.hex() == r
            assert S.compute_signing_root(root, bytes.fromhex(d)).hex() == sr


def test_oracle_bitlist_and_zero_padding():
    # an empty list's root is the zero subtree of its limit mixed with length 0
    assert S.mix_in_length(S.merkleize([], 16), 0) == S.H(S.merkleize([], 16) + bytes(32))
    # a bitlist of 3 set bits: serialized 0b1111 (delimiter at bit 3)
    assert S.bitlist_root(bytes([0x0F]), 2048) == S.mix_in_length(S.merkleize([bytes([0x07]) + bytes(31)], 8), 3)


def test_host_serializers_match_oracle_layout():
    from lodestar_amd import ssz

    a = ssz.serialize_attestation_data(5, 2, b"\x01" * 32, 3, b"\x02" * 32, 4, b"\x03" * 32)
    assert a == S.ser_attestation_data(5, 2, b"\x01" * 32, 3, b"\x02" * 32, 4, b"\x03" * 32)
    h = ssz.serialize_beacon_block_header(1, 2, b"\x04" * 32, b"\x05" * 32, b"\x06" * 32)
    assert h == S.ser_header(1, 2, b"\x04" * 32, b"\x05" * 32, b"\x06" * 32)
    with pytest.raises(ValueError):
        ssz.serialize_attestation_data(0, 0, b"\x00" * 31, 0, b"\x00" * 32, 0, b"\x00" * 32)


# ----------------------------------------------------------------------------- GPU
def _att_data_bytes(d: dict) -> bytes:
    h = lambda s: bytes.fromhex(s[2:])  # noqa: E731
    return S.ser_attestation_data(int(d["slot"]), int(d["index"]), h(d["beacon_block_root"]),
                                  int(d["source"]["epoch"]), h(d["source"]["root"]),
                                  int(d["target"]["epoch"]), h(d["target"]["root"]))


@pytest.mark.gpu
def test_gpu_vectors_every_kind(gpu):
    from lodestar_amd import ssz

    for kind, v in G["vectors"].items():
        objs = b"".join(bytes.fromhex(o) for o in v["objs"])
        roots = ssz.hash_tree_roots(gpu, kind, objs)
        assert [r.tobytes().hex() for r in roots] == v["roots"], kind
        doms = b"".join(bytes.fromhex(d) for d in v["domains"])
        sroots = ssz.compute_signing_roots(gpu, kind, objs, doms)
        assert [r.tobytes().hex() for r in sroots] == v["signing_roots"], kind
        # one shared domain (stride 0)
        one = ssz.compute_signing_roots(gpu, kind, objs, bytes.fromhex(v["domains"][0]))
        want = [S.compute_signing_root(bytes.fromhex(r), bytes.fromhex(v["domains"][0])).hex() for r in v["roots"]]
        assert [r.tobytes().hex() for r in one] == want, kind


@pytest.mark.gpu
def test_gpu_mainnet_block_chain(gpu):
    """GPU AttestationData roots of the 45 mainnet attestations feed the body roots, then
    GPU header roots must equal the next blocks' parent roots."""
    from lodestar_amd import ssz

    for blk, want in zip(G["blocks"], G["expected_roots"]):
        atts = blk["body"]["attestations"]
        data_roots = []
        if atts:
            rs = ssz.hash_tree_roots(gpu, "attestation_data", [_att_data_bytes(a["data"]) for a in atts])
            data_roots = [r.tobytes() for r in rs]
            assert data_roots == [S.attestation_data_json_root(a["data"]) for a in atts]
        body_root = S.body_json_root_phase0(blk["body"], data_roots or None)
        hdr = ssz.serialize_beacon_block_header(int(blk["slot"]), int(blk["proposer_index"]),
                                                bytes.fromhex(blk["parent_root"][2:]),
                                                bytes.fromhex(blk["state_root"][2:]), body_root)
        assert ssz.hash_tree_roots(gpu, "beacon_block_header", hdr)[0].tobytes().hex() == want


@pytest.mark.gpu
def test_gpu_kat1_deposit_signing_root(gpu):
    from lodestar_amd import ssz

    k = G["kat1_deposit"]
    dom = ssz.compute_domain(gpu, ssz.DOMAIN_DEPOSIT, bytes.fromhex(k["fork_version"]),
                             bytes.fromhex(k["genesis_validators_root"]))
    assert dom.hex() == k["domain"]
    msg = ssz.serialize_deposit_message(bytes.fromhex(k["pubkey"]), bytes.fromhex(k["withdrawal_credentials"]),
                                        k["amount"])
    assert ssz.compute_signing_root(gpu, "deposit_message", msg, dom).hex() == k["signing_root"]


@pytest.mark.gpu
def test_gpu_epoch_of_attestations_and_edges(gpu):
    """A mainnet epoch's attestation-data shape (2048 committees, 32 slots) in one launch,
    an empty batch, and an unknown kind."""
    import random

    from lodestar_amd import ssz
    from lodestar_amd.native import NativeError

    rng = random.Random(7)
    roots = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(34)]
    datas = [S.ser_attestation_data(s, c, roots[s], 9, roots[32], 10, roots[33]) for s in range(32) for c in range(64)]
    dom = bytes(rng.getrandbits(8) for _ in range(32))
    got = ssz.compute_signing_roots(gpu, "attestation_data", datas, dom)
    for i in rng.sample(range(len(datas)), 64):
        want = S.compute_signing_root(S.root_of_serialized("attestation_data", datas[i]), dom)
        assert got[i].tobytes() == want
    assert gpu.ssz_roots(ssz.KINDS["uint64"], b"", None).shape == (0, 32)
    with pytest.raises(NativeError):
        gpu.ssz_roots(0x900 | 8, bytes(8), None)
