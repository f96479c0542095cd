"""State-transition inline signature checks on the GPU.

When block signatures are not batch-verified, the state transition verifies sets one
by one with `verifySignatureSet` (state-transition/src/util/signatureSets.ts:24-38),
called from block/processAttestationsAltair.ts:56, block/processProposerSlashing.ts:61,
block/isValidIndexedAttestation.ts:20,36, block/processSyncCommittee.ts:31 and the
signatureSets/{randao,proposer,voluntaryExits}.ts helpers.  The reference semantics:

* `Signature.fromBytes(sig, undefined, validate=true)` -- a signature that does not
  decode or lies outside G2 throws;
* single set: `signature.verify(pubkey, signingRoot)`; aggregate set:
  `signature.verifyAggregate(pubkeys, signingRoot)` (the pubkeys summed first,
  `PublicKey.aggregate`, which throws on an empty list).

Here each set is one non-batchable request of one set through bls_gpu_verify (the
1-set path of verifySignatureSetsMaybeBatch, maybeBatch.ts:33-38), run at once on the
caller's thread -- no buffering, like the reference's synchronous call.  Several inline
checks of one block can go in ONE GPU call (`verify_signature_sets_each`) with each set
keeping its own verdict.
"""
from __future__ import annotations

from typing import Sequence

from .native import GpuContext, pack_requests
from .verifier import BlsError, SignatureSet, _wire



def _settle(code: int) -> bool:
    from ._abi import ERROR_MESSAGES

    if code < 0:
        raise BlsError(ERROR_MESSAGES.get(-code, f"BLST_ERROR: {-code}"))
    return code == 1


def verify_signature_set(ctx: GpuContext, s: SignatureSet) -> bool:
    """verifySignatureSet (signatureSets.ts:24-38) for one set: True / False, or raises
    BlsError with the blst-style message when the signature (or the aggregate) fails."""
    v, _ = ctx.verify_packed(pack_requests([(False, [_wire(s)])]))
    return _settle(int(v[0]))


def verify_signature_sets_each(ctx: GpuContext, sets: Sequence[SignatureSet]) -> list:
    """verifySignatureSet for each of `sets` in one GPU call: a list of True / False or
    BlsError (the exception the set's own verifySignatureSet would raise)."""
    if not sets:
        return []
    v, _ = ctx.verify_packed(pack_requests([(False, [_wire(s)]) for s in sets]))
    out = []
    for code in v:
        try:
            out.append(_settle(int(code)))
        except BlsError as e:
            out.append(e)
    return out
