"""Signing roots on the GPU: the step before the verify path.

Mirrors the reference's helpers with the same names and argument meaning:

* `compute_signing_root(gpu, kind, obj, domain)`  -- computeSigningRoot(type, sszObject,
  domain) (`state-transition/src/util/signingRoot.ts:7-13`), `kind` standing for the
  SSZ type;
* `compute_signing_roots(gpu, kind, objs, domains)` -- the same over a batch (the
  producers in `state-transition/src/signatureSets/*.ts` build one per set; a block's or
  an epoch's worth of attestations go through one launch);
* `compute_fork_data_root` / `compute_domain` (`state-transition/src/util/domain.ts:9-45`).

Objects are passed in their SSZ serialization (the `serialize_*` helpers build it from
field values).  Every root is computed by `k_ssz_roots` (bls_gpu_ssz_roots); there is no
CPU path.
"""
from __future__ import annotations

import numpy as np

from . import _abi as A

KINDS = {
    "root": A.SSZ_ROOT,
    "uint64": A.SSZ_UINT64,
    "checkpoint": A.SSZ_CHECKPOINT,
    "attestation_data": A.SSZ_ATTESTATION_DATA,
    "two_uint64": A.SSZ_TWO_UINT64,
    "voluntary_exit": A.SSZ_TWO_UINT64,
    "sync_aggregator_selection_data": A.SSZ_TWO_UINT64,
    "beacon_block_header": A.SSZ_BEACON_BLOCK_HEADER,
    "deposit_message": A.SSZ_DEPOSIT_MESSAGE,
    "fork_data": A.SSZ_FORK_DATA,
    "signing_data": A.SSZ_SIGNING_DATA,
}

# DomainType values (params/src/index.ts:110-119)
DOMAIN_BEACON_PROPOSER = bytes.fromhex("00000000")
DOMAIN_BEACON_ATTESTER = bytes.fromhex("01000000")
DOMAIN_RANDAO = bytes.fromhex("02000000")
DOMAIN_DEPOSIT = bytes.fromhex("03000000")
DOMAIN_VOLUNTARY_EXIT = bytes.fromhex("04000000")
DOMAIN_SELECTION_PROOF = bytes.fromhex("05000000")
DOMAIN_AGGREGATE_AND_PROOF = bytes.fromhex("06000000")
DOMAIN_SYNC_COMMITTEE = bytes.fromhex("07000000")
DOMAIN_SYNC_COMMITTEE_SELECTION_PROOF = bytes.fromhex("08000000")
DOMAIN_CONTRIBUTION_AND_PROOF = bytes.fromhex("09000000")


def _kind(kind) -> int:
    return KINDS[kind] if isinstance(kind, str) else int(kind)


def _b32(b: bytes, what: str) -> bytes:
    b = bytes(b)
    if len(b) != 32:
        raise ValueError(f"{what} must be 32 bytes, got {len(b)}")
    return b


def _u64(v: int) -> bytes:
    return int(v).to_bytes(8, "little")


# ---- SSZ serializations of the fixed-size kinds ------------------------------------
def serialize_attestation_data(slot: int, index: int, beacon_block_root: bytes, source_epoch: int,
                               source_root: bytes, target_epoch: int, target_root: bytes) -> bytes:
    return (_u64(slot) + _u64(index) + _b32(beacon_block_root, "beacon_block_root") + _u64(source_epoch)
            + _b32(source_root, "source.root") + _u64(target_epoch) + _b32(target_root, "target.root"))


def serialize_beacon_block_header(slot: int, proposer_index: int, parent_root: bytes, state_root: bytes,
                                  body_root: bytes) -> bytes:
    return (_u64(slot) + _u64(proposer_index) + _b32(parent_root, "parent_root") + _b32(state_root, "state_root")
            + _b32(body_root, "body_root"))


def serialize_voluntary_exit(epoch: int, validator_index: int) -> bytes:
    return _u64(epoch) + _u64(validator_index)


def serialize_deposit_message(pubkey48: bytes, withdrawal_credentials: bytes, amount: int) -> bytes:
    if len(pubkey48) != 48:
        raise ValueError("pubkey must be 48 bytes")
    return bytes(pubkey48) + _b32(withdrawal_credentials, "withdrawal_credentials") + _u64(amount)


def serialize_uint64(v: int) -> bytes:
    return _u64(v)


# ---- the reference's helpers ----------------------------------------------------------
def compute_signing_roots(gpu, kind, objs, domains) -> np.ndarray:
    """n x 32 signing roots of n serialized objects (bytes, or a list of per-object
    bytes); domains: one 32-byte domain or one per object."""
    if isinstance(objs, (list, tuple)):
        objs = b"".join(objs)
    if isinstance(domains, (list, tuple)):
        domains = b"".join(domains)
    return gpu.ssz_roots(_kind(kind), objs, domains)


def compute_signing_root(gpu, kind, obj: bytes, domain: bytes) -> bytes:
    """computeSigningRoot(type, sszObject, domain) (signingRoot.ts:7-13)."""
    return compute_signing_roots(gpu, kind, obj, _b32(domain, "domain"))[0].tobytes()


def hash_tree_roots(gpu, kind, objs) -> np.ndarray:
    """type.hashTreeRoot for a batch of serialized objects."""
    if isinstance(objs, (list, tuple)):
        objs = b"".join(objs)
    return gpu.ssz_roots(_kind(kind), objs, None)


def compute_fork_data_root(gpu, current_version: bytes, genesis_validators_root: bytes) -> bytes:
    """computeForkDataRoot (domain.ts:40-45)."""
    if len(current_version) != 4:
        raise ValueError("fork version must be 4 bytes")
    obj = bytes(current_version) + _b32(genesis_validators_root, "genesis_validators_root")
    return gpu.ssz_roots(A.SSZ_FORK_DATA, obj, None)[0].tobytes()


def compute_domain(gpu, domain_type: bytes, fork_version: bytes, genesis_validators_root: bytes) -> bytes:
    """computeDomain (domain.ts:9-16): domain_type || fork_data_root[:28]."""
    if len(domain_type) != 4:
        raise ValueError("domain type must be 4 bytes")
    return bytes(domain_type) + compute_fork_data_root(gpu, fork_version, genesis_validators_root)[:28]
