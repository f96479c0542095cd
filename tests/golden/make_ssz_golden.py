#!/usr/bin/env python3
"""Generate tests/golden/ssz_golden.json: SSZ signing-root fixtures (build container only;
the JSON is committed and is all the GPU box reads).

    python tests/golden/make_ssz_golden.py

* `blocks`: the 4 mainnet phase0 blocks of the reference's backfill-sync fixture
  (packages/beacon-node/test/unit/sync/backfill/blocks.json, data copied as a fixture),
  with `expected_roots[i]` = blocks[i + 1].parent_root -- the chain
  sync/backfill/verify.ts checks.  The oracle (oracle/ssz_oracle.py) must reproduce
  them before anything else here is trusted.
* `kat1_deposit`: KAT-1's deposit message and signing root (genesisState.test.ts:65-69,
  minimal preset GENESIS_FORK_VERSION 0x00000001, zero genesis_validators_root).
* `vectors`: seeded random objects of every kernel kind with the oracle's
  hash_tree_root and signing root.
"""
from __future__ import annotations

import json
import random
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import ssz_oracle as S  # noqa: E402

BLOCKS = Path("/root/reference/packages/beacon-node/test/unit/sync/backfill/blocks.json")
SIZES = {"root": 32, "uint64": 8, "checkpoint": 40, "attestation_data": 128, "two_uint64": 16,
         "beacon_block_header": 112, "deposit_message": 88, "fork_data": 36, "signing_data": 64}


def main() -> None:
    blocks = [b["message"] for b in json.loads(BLOCKS.read_text())]
    expected = [blocks[i + 1]["parent_root"][2:] for i in range(len(blocks) - 1)]
    for i, e in enumerate(expected):
        assert S.block_json_root_phase0(blocks[i]).hex() == e, f"oracle disagrees with mainnet block {i}"
    out: dict = {"source": "packages/beacon-node/test/unit/sync/backfill/blocks.json (mainnet slots 1-4)",
                 "blocks": blocks, "expected_roots": expected}

    pk0 = bytes.fromhex("a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c")
    wc0 = bytes.fromhex("00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b")
    amount = 32_000_000_000
    domain = S.compute_domain(bytes.fromhex("03000000"), bytes.fromhex("00000001"), bytes(32))
    root = S.compute_signing_root(S.deposit_message_root(pk0, wc0, amount), domain)
    golden = json.loads((HERE / "golden.json").read_text())
    assert root.hex() == golden["kat1"]["signing_root"], "KAT-1 signing root"
    out["kat1_deposit"] = {"pubkey": pk0.hex(), "withdrawal_credentials": wc0.hex(), "amount": amount,
                           "fork_version": "00000001", "genesis_validators_root": "00" * 32,
                           "domain": domain.hex(), "signing_root": root.hex(),
                           "source": "genesisState.test.ts:65-69 (minimal preset)"}

    rng = random.Random(0x5510)
    vec = {}
    for kind, size in SIZES.items():
        objs = [bytes(rng.getrandbits(8) for _ in range(size)) for _ in range(16)]
        doms = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(16)]
        vec[kind] = {"objs": [o.hex() for o in objs], "domains": [d.hex() for d in doms],
                     "roots": [S.root_of_serialized(kind, o).hex() for o in objs],
                     "signing_roots": [S.compute_signing_root(S.root_of_serialized(kind, o), d).hex()
                                       for o, d in zip(objs, doms)]}
    out["vectors"] = vec
    (HERE / "ssz_golden.json").write_text(json.dumps(out, indent=1) + "\n")
    print("wrote", HERE / "ssz_golden.json")


if __name__ == "__main__":
    main()
