#!/usr/bin/env python3
"""Generate tests/golden/*.json from the CPU oracle (oracle/bls_oracle.py) and the
reference's own in-repo known-answer data.  Run in the build container only
(needs /root/reference for the KAT sources); the JSON outputs are committed and are
all the GPU box ever reads.

    python tests/golden/make_golden.py

Reference data copied as fixture values (data, not source):
  * KAT-1  interop deposit #0: pubkey / withdrawal credentials / signature
           (packages/beacon-node/test/e2e/interop/genesisState.test.ts:65-69).  The test runs
           under the minimal preset (test/setupPreset.ts:2-3), GENESIS_FORK_VERSION 0x00000001
           (config/src/chainConfig/presets/minimal.ts:23); the signing root is derived below.
  * KAT-2  100 interop pubkeys (packages/state-transition/test-cache/interop-pubkeys.json).
  * KAT-3  real mainnet G2 points (packages/beacon-node/test/unit/sync/backfill/blocks.json,
           randao_reveal + signature), the "valid signature of random data"
           (beacon-node/test/unit/chain/opPools/aggregatedAttestationPool.test.ts:22-24) and the
           two selection proofs of state-transition/test/unit/util/aggregator.test.ts:28,37.
           The "bruteforced" invalid signature of aggregator.test.ts:70 goes to
           kat3_unpinned with the oracle's decode code: the reference test only hashes it, so
           its decode outcome is parity unpinned.
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import bls_oracle as O  # noqa: E402

REF = Path("/root/reference/packages")


def H(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def deposit_signing_root(pk: bytes, wc: bytes, amount: int, fork_version: bytes) -> bytes:
    """SSZ hash_tree_root(SigningData{hash_tree_root(DepositMessage), domain}) with
    domain = DOMAIN_DEPOSIT || fork_data_root[:28], zero genesis_validators_root."""
    amount_chunk = amount.to_bytes(8, "little") + bytes(24)
    obj = H(H(H(pk + bytes(16)) + wc) + H(amount_chunk + bytes(32)))
    fork_data_root = H(fork_version + bytes(28) + bytes(32))
    domain = bytes.fromhex("03000000") + fork_data_root[:28]
    return H(obj + domain)


def g2_uncompressed(pt) -> str:
    if pt is None:
        return (bytes([0x40]) + bytes(191)).hex()
    (x0, x1), (y0, y1) = pt
    return b"".join(v.to_bytes(48, "big") for v in (x1, x0, y1, y0)).hex()


def main() -> None:
    out: dict = {}
    # ---- KAT-1
    pk0 = bytes.fromhex("a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c")
    wc0 = bytes.fromhex("00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b")
    sig0 = bytes.fromhex(
        "a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
        "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446")
    root0 = deposit_signing_root(pk0, wc0, 32_000_000_000, bytes.fromhex("00000001"))
    out["kat1"] = {"sk": "%064x" % O.interop_secret_key(0), "pubkey": pk0.hex(), "signing_root": root0.hex(),
                   "signature": sig0.hex(), "source": "genesisState.test.ts:65-69 (minimal preset)"}
    # ---- KAT-2
    pubs = json.loads((REF / "state-transition/test-cache/interop-pubkeys.json").read_text())
    out["kat2_interop_pubkeys"] = [p[2:] if p.startswith("0x") else p for p in pubs]
    # ---- KAT-3
    blocks = json.loads((REF / "beacon-node/test/unit/sync/backfill/blocks.json").read_text())
    g2 = []
    for b in blocks:
        g2.append(b["message"]["body"]["randao_reveal"][2:])
        g2.append(b["signature"][2:])
    g2.append("b2afb700f6c561ce5e1b4fedaec9d7c06b822d38c720cf588adfda748860a940adf51634b6788f298c552de40183b5a2"
              "03b2bbe8b7dd147f0bb5bc97080a12efbb631c8888cb31a99cc4706eb3711865b8ea818c10126e4d818b542e9dbf9ae8")
    # aggregator.test.ts:28,37: selection proofs (valid G2 points)
    agg_src = (REF / "state-transition/test/unit/util/aggregator.test.ts").read_text()
    agg_hex = [h for h in (ln.strip().strip('"') for ln in agg_src.splitlines()) if h.startswith("0x") and len(h) == 194]
    assert len(agg_hex) == 4, "aggregator.test.ts: four 96-byte hex literals expected"
    g2 += [agg_hex[0][2:], agg_hex[1][2:]]
    out["kat3_g2_points"] = [{"compressed": h, "uncompressed": g2_uncompressed(O.signature_from_bytes(bytes.fromhex(h)))}
                             for h in g2]
    # aggregator.test.ts:70 (":68 NOTE: Invalid sig, bruteforced last characters"): the oracle's
    # decode code, parity unpinned (the reference never decodes it)
    unp = []
    for h in (agg_hex[3][2:],):
        try:
            O.signature_from_bytes(bytes.fromhex(h), validate=True)
            code = 0
        except O.BlsError as e:
            code = e.code
        unp.append({"compressed": h, "code": code, "source": "aggregator.test.ts:70", "parity": "unpinned"})
    out["kat3_unpinned"] = unp

    # ---- oracle-derived vectors (pinned by KAT-1/2/3 above)
    sks = [O.interop_secret_key(i) for i in range(8)]
    msgs = [H(b"lodestar-amd golden %d" % j) for j in range(6)] + [bytes(32), b"\xff" * 32]
    out["hash_to_g2"] = [{"msg": m.hex(), "point": g2_uncompressed(O.hash_to_g2(m))} for m in msgs]
    pk_pts = [O.sk_to_pk(s) for s in sks]
    agg_lists = [[0], [0, 1], [2, 3, 4], list(range(8)), [5, 5], [7, 0, 3]]
    out["aggregate"] = {"sks": ["%064x" % s for s in sks],
                        "lists": agg_lists,
                        "expected": [O.g1_serialize(O.aggregate_pubkeys([pk_pts[i] for i in L])).hex()
                                     for L in agg_lists]}
    sigs = []
    for i in range(4):
        for j in range(2):
            sigs.append({"sk": "%064x" % sks[i], "msg": msgs[j].hex(), "sig": O.g2_compress(O.sign(sks[i], msgs[j])).hex()})
    out["signatures"] = sigs
    # decoding edge cases (spec-derived; parity unpinned by reference tests beyond KAT-3/4)
    valid = bytes.fromhex(sigs[0]["sig"])
    cases = {
        "valid": valid,
        "infinity": bytes([0xC0]) + bytes(95),
        "infinity_bad_flag": bytes([0xE0]) + bytes(95),
        "no_compression_flag": bytes([valid[0] & 0x7F]) + valid[1:],
        "x_ge_p": bytes([0x80 | 0x1A, 0x01, 0x11, 0xEA]) + b"\xff" * 92,
    }
    # an x with no curve point, and a point on E2 outside G2
    x1 = 1
    while True:
        b = bytearray(96)
        b[0] = 0x80
        b[95] = x1
        code, pt = O.g2_decompress(bytes(b))
        if code == O.E_POINT_NOT_ON_CURVE and "not_on_curve" not in cases:
            cases["not_on_curve"] = bytes(b)
        if code == O.E_OK and pt is not None and not O.g2_in_subgroup(pt) and "not_in_group" not in cases:
            cases["not_in_group"] = bytes(b)
        if "not_on_curve" in cases and "not_in_group" in cases:
            break
        x1 += 1
    dec = []
    for name, raw in cases.items():
        try:
            O.signature_from_bytes(raw, validate=True)
            code = 0
        except O.BlsError as e:
            code = e.code
        dec.append({"name": name, "bytes": raw.hex(), "code": code})
    out["sig_decode"] = dec
    (HERE / "golden.json").write_text(json.dumps(out, indent=1) + "\n")
    print("wrote", HERE / "golden.json")


if __name__ == "__main__":
    main()
