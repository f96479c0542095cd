"""G2 signature aggregation and the light client's aggregate check on the GPU
(SURVEY.md §8f rank 4).

* Op pools aggregate attestation / sync-committee signatures for block production:
  `bls.Signature.aggregate(sigs.map((s) => bls.Signature.fromBytes(s, undefined, true)))`
  (beacon-node/src/chain/opPools/aggregatedAttestationPool.ts:320-327 aggregateInto,
  syncContributionAndProofPool.ts:181-185, syncCommitteeMessagePool.ts:122-129) ->
  `signature_aggregate` (bls_gpu_aggregate_signatures: per signature decode + G2
  membership, per list the sum, compressed).
* The light client checks a sync aggregate with `isValidBlsAggregate(pubkeys,
  signingRoot, signature)` (light-client/src/validation.ts:167-190): aggregate the
  participants' keys, decode the signature with validation, verify ->
  `is_valid_bls_aggregate`: an aggregate set over device-table indices (the sync
  committee's keys loaded once per period, pubkeyCache-style), one non-batchable
  request, so the 1-set rules apply as in Signature.verify.
"""
from __future__ import annotations

from typing import Sequence

from .native import GpuContext, pack_requests
from .verifier import BlsError


def _raise(code: int, what: str):
    from ._abi import ERROR_MESSAGES

    raise BlsError(f"{what}: " + ERROR_MESSAGES.get(code, f"BLST_ERROR: {code}"))


def signature_aggregate(ctx: GpuContext, sig_lists: Sequence[Sequence[bytes]]) -> list[bytes]:
    """Signature.aggregate of each list (96-byte compressed signatures, each decoded with
    validate=true); raises BlsError for a list with an undecodable / out-of-group
    signature or an empty list (EMPTY_AGGREGATE_ARRAY)."""
    out, codes = ctx.aggregate_signatures(sig_lists)
    for k, c in enumerate(codes):
        if c != 0:
            _raise(int(c), f"aggregating list {k}")
    return out


def aggregate_into(ctx: GpuContext, sig1: bytes, sig2: bytes) -> bytes:
    """aggregateInto's signature part (aggregatedAttestationPool.ts:320-327)."""
    return signature_aggregate(ctx, [[sig1, sig2]])[0]


def is_valid_bls_aggregate(ctx: GpuContext, pubkey_indices: Sequence[int], message: bytes, signature: bytes) -> bool:
    """isValidBlsAggregate (light-client/src/validation.ts:167-190) over keys already in
    the context's device table: True / False; raises BlsError when the keys do not
    aggregate (empty list) or the signature does not decode."""
    v, _ = ctx.verify_packed(pack_requests([(False, [(list(pubkey_indices), bytes(message), bytes(signature))])]))
    code = int(v[0])
    if code < 0:
        _raise(-code, "isValidBlsAggregate")
    return code == 1
