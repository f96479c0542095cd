"""CPU ORACLE for SSZ signing roots — test infrastructure only, never on the product path.

Restates the SSZ merkleization the reference reaches through `@chainsafe/ssz`
(un-vendored npm dependency, `yarn.lock`; absent from /root/reference) for the
fixed-size containers whose signing roots feed the BLS verify path:

* `computeSigningRoot(type, obj, domain)` = hash_tree_root(SigningData{objectRoot,
  domain}) (`state-transition/src/util/signingRoot.ts:7-13`);
* `computeDomain` / `computeForkDataRoot` (`state-transition/src/util/domain.ts:9-45`);
* the signature-set producers' object types: AttestationData
  (`signatureSets/indexedAttestation.ts:17-24`), Epoch (`randao.ts:26-31`), the block
  header / block (`proposer.ts:23-33`), VoluntaryExit (`voluntaryExits.ts:27-33`),
  DepositMessage (`block/processDeposit.ts`), SyncAggregatorSelectionData, Root (sync
  committee messages).

Merkleization follows the SSZ spec (consensus-specs ssz/simple-serialize.md): basic
values packed little-endian into 32-byte chunks, containers = merkleize(field roots)
padded to the next power of two with zero chunks, lists / bitlists mixed in with
their length.  Phase 0 mainnet limits are used for the BeaconBlockBody lists.

Pinned by reference-held data (tests/test_ssz.py): the 4 mainnet blocks of
`beacon-node/test/unit/sync/backfill/blocks.json` — hash_tree_root(block i) must equal
block i+1's parent_root (what `sync/backfill/verify.ts` checks), which covers
AttestationData, Checkpoint, Bitlist, BLSSignature, Eth1Data, the body lists and the
header; and KAT-1, the interop deposit signing root
(`beacon-node/test/e2e/interop/genesisState.test.ts:65-69`).
"""
from __future__ import annotations

import hashlib

ZERO = bytes(32)

# phase0 mainnet limits (params/src/presets/mainnet/phase0.ts)
MAX_VALIDATORS_PER_COMMITTEE = 2048
MAX_PROPOSER_SLASHINGS = 16
MAX_ATTESTER_SLASHINGS = 2
MAX_ATTESTATIONS = 128
MAX_DEPOSITS = 16
MAX_VOLUNTARY_EXITS = 16


def H(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def chunk(b: bytes) -> bytes:
    assert len(b) <= 32
    return b + bytes(32 - len(b))


def uint64(v: int) -> bytes:
    return chunk(int(v).to_bytes(8, "little"))


def _next_pow2(n: int) -> int:
    p = 1
    while p < n:
        p *= 2
    return p


def merkleize(chunks: list[bytes], limit: int | None = None) -> bytes:
    """merkleize(chunks, limit): pad to next_pow2(limit or len) leaves with zero chunks."""
    width = _next_pow2(max(1, limit if limit is not None else len(chunks)))
    assert len(chunks) <= width
    zero = ZERO
    layer = list(chunks)
    while width > 1:
        if len(layer) % 2:
            layer.append(zero)
        layer = [H(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
        zero = H(zero + zero)
        width //= 2
    return layer[0] if layer else zero


def mix_in_length(root: bytes, length: int) -> bytes:
    return H(root + length.to_bytes(32, "little"))


def bytes_root(b: bytes) -> bytes:
    """ByteVector[N]: packed into ceil(N/32) chunks."""
    return merkleize([chunk(b[i:i + 32]) for i in range(0, len(b), 32)])


def bitlist_root(serialized: bytes, limit: int) -> bytes:
    """Bitlist[limit] from its SSZ serialization (delimiter bit = the last byte's top set bit)."""
    last = serialized[-1]
    assert last != 0, "bitlist without delimiter"
    top = last.bit_length() - 1
    n_bits = 8 * (len(serialized) - 1) + top
    data = bytearray(serialized)
    data[-1] &= ~(1 << top) & 0xFF
    n_bytes = (n_bits + 7) // 8
    data = bytes(data[:n_bytes])
    chunks = [chunk(data[i:i + 32]) for i in range(0, len(data), 32)]
    return mix_in_length(merkleize(chunks, (limit + 255) // 256), n_bits)


# ---- fixed-size containers (field values as python ints / bytes) -------------------
def checkpoint_root(epoch: int, root: bytes) -> bytes:
    return merkleize([uint64(epoch), root])


def attestation_data_root(slot, index, beacon_block_root, source_epoch, source_root, target_epoch, target_root) -> bytes:
    return merkleize([uint64(slot), uint64(index), beacon_block_root, checkpoint_root(source_epoch, source_root),
                      checkpoint_root(target_epoch, target_root)])


def beacon_block_header_root(slot, proposer_index, parent_root, state_root, body_root) -> bytes:
    return merkleize([uint64(slot), uint64(proposer_index), parent_root, state_root, body_root])


def deposit_message_root(pubkey48: bytes, withdrawal_credentials: bytes, amount: int) -> bytes:
    return merkleize([bytes_root(pubkey48), withdrawal_credentials, uint64(amount)])


def two_uint64_root(a: int, b: int) -> bytes:
    """VoluntaryExit{epoch, validator_index}, SyncAggregatorSelectionData{slot, subcommittee_index}."""
    return merkleize([uint64(a), uint64(b)])


def fork_data_root(current_version: bytes, genesis_validators_root: bytes) -> bytes:
    return merkleize([chunk(current_version), genesis_validators_root])


def compute_domain(domain_type: bytes, fork_version: bytes, genesis_validators_root: bytes) -> bytes:
    """domain.ts:9-16: domain_type (4) || fork_data_root[:28]."""
    return domain_type + fork_data_root(fork_version, genesis_validators_root)[:28]


def compute_signing_root(object_root: bytes, domain: bytes) -> bytes:
    """signingRoot.ts:7-13: hash_tree_root(SigningData{object_root, domain})."""
    return merkleize([object_root, domain])


# ---- SSZ serializations of the fixed-size kinds (the GPU kernel's input layout) -----
def ser_u64(v: int) -> bytes:
    return int(v).to_bytes(8, "little")


def ser_attestation_data(slot, index, bbr, se, sr, te, tr) -> bytes:
    return ser_u64(slot) + ser_u64(index) + bbr + ser_u64(se) + sr + ser_u64(te) + tr


def ser_header(slot, proposer_index, parent_root, state_root, body_root) -> bytes:
    return ser_u64(slot) + ser_u64(proposer_index) + parent_root + state_root + body_root


def root_of_serialized(kind: str, obj: bytes) -> bytes:
    """hash_tree_root of one serialized object of `kind` (the GPU kernel's kinds)."""
    u = lambda off: int.from_bytes(obj[off:off + 8], "little")  # noqa: E731
    if kind == "root":
        return obj[:32]
    if kind == "uint64":
        return uint64(u(0))
    if kind == "checkpoint":
        return checkpoint_root(u(0), obj[8:40])
    if kind == "attestation_data":
        return attestation_data_root(u(0), u(8), obj[16:48], u(48), obj[56:88], u(88), obj[96:128])
    if kind == "two_uint64":
        return two_uint64_root(u(0), u(8))
    if kind == "beacon_block_header":
        return beacon_block_header_root(u(0), u(8), obj[16:48], obj[48:80], obj[80:112])
    if kind == "deposit_message":
        return deposit_message_root(obj[:48], obj[48:80], u(80))
    if kind == "fork_data":
        return fork_data_root(obj[:4], obj[4:36])
    if kind == "signing_data":
        return compute_signing_root(obj[:32], obj[32:64])
    raise ValueError(kind)


# ---- phase0 block (JSON as in blocks.json) -------------------------------------------
def _h(s: str) -> bytes:
    return bytes.fromhex(s[2:] if s.startswith("0x") else s)


def attestation_data_json_root(d: dict) -> bytes:
    return attestation_data_root(int(d["slot"]), int(d["index"]), _h(d["beacon_block_root"]),
                                 int(d["source"]["epoch"]), _h(d["source"]["root"]),
                                 int(d["target"]["epoch"]), _h(d["target"]["root"]))


def attestation_json_root(a: dict, data_root: bytes | None = None) -> bytes:
    """Attestation{aggregation_bits: Bitlist[2048], data, signature: BLSSignature}."""
    return merkleize([bitlist_root(_h(a["aggregation_bits"]), MAX_VALIDATORS_PER_COMMITTEE),
                      data_root if data_root is not None else attestation_data_json_root(a["data"]),
                      bytes_root(_h(a["signature"]))])


def body_json_root_phase0(body: dict, attestation_data_roots: list[bytes] | None = None) -> bytes:
    """phase0 BeaconBlockBody; only empty slashing / deposit / exit lists are handled
    (the blocks.json fixture has none)."""
    for k in ("proposer_slashings", "attester_slashings", "deposits", "voluntary_exits"):
        assert not body[k], f"{k} not supported by this oracle"
    e = body["eth1_data"]
    eth1 = merkleize([_h(e["deposit_root"]), uint64(int(e["deposit_count"])), _h(e["block_hash"])])
    atts = body["attestations"]
    roots = [attestation_json_root(a, attestation_data_roots[i] if attestation_data_roots else None)
             for i, a in enumerate(atts)]
    return merkleize([
        bytes_root(_h(body["randao_reveal"])),
        eth1,
        _h(body["graffiti"]),
        mix_in_length(merkleize([], MAX_PROPOSER_SLASHINGS), 0),
        mix_in_length(merkleize([], MAX_ATTESTER_SLASHINGS), 0),
        mix_in_length(merkleize(roots, MAX_ATTESTATIONS), len(roots)),
        mix_in_length(merkleize([], MAX_DEPOSITS), 0),
        mix_in_length(merkleize([], MAX_VOLUNTARY_EXITS), 0),
    ])


def block_json_root_phase0(msg: dict) -> bytes:
    return beacon_block_header_root(int(msg["slot"]), int(msg["proposer_index"]), _h(msg["parent_root"]),
                                    _h(msg["state_root"]), body_json_root_phase0(msg["body"]))
