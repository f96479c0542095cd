"""Synthetic inputs of BASELINE.json's configs, shared by bench.py and
the GPU parity tests.  Nothing here verifies anything: keys, messages and signatures
are made with the library's own fixture helpers (bls_gpu_sk_to_pk / bls_gpu_sign,
pinned bit-exact against the oracle by tests/test_gpu_parity.py), and the validity of
every set is known by construction.

* keys: interop secret keys sk_i = LE(sha256(LE32(i))) mod r
  (state-transition/src/util/interop.ts:19-22), a device pubkey table of `n_keys`
  (Index2PubkeyCache, pubkeyCache.ts:56-77; 1M keys ~ the mainnet validator set);
* messages: m_j = sha256(LE64(j) || tag), distinct per set (cfg1-4) or shared per
  committee (cfg5);
* an aggregate set signs with sum_k sk_k (its signature is the aggregate of its
  members' signatures, the sets getIndexedAttestationSignatureSet builds,
  state-transition/src/signatureSets/indexedAttestation.ts:6-28).

cfg3 (one block import, CS-2): 128 aggregate sets x 512 distinct keys sampled without
replacement from the table (seed 1) with 128 distinct roots, plus the sync-committee
aggregate of 512 keys -- one non-batchable request of 129 sets
(verifyBlock.ts:183-190 -> chunkifyMaximizeChunkSize(sets, 128) gives one job).

cfg4 (range-sync replay): 90 % single / 10 % aggregate (k = 128) sets, 1 % invalid
chosen uniformly (seed 2; half signed over another message, half by another key),
grouped into calls of 128 sets; call c goes to GPU c mod world (shard by call).

cfg5 (mainnet epoch shape): single-pubkey attestations over committees of
`n_sets / n_roots` consecutive sets sharing one signing root (2048 roots per epoch,
256 per GPU of 8), calls of 1024 batchable single-set requests (gossip, CS-1).
"""
from __future__ import annotations

import hashlib
import random
from dataclasses import dataclass, field

import numpy as np

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

_SK_CACHE: list[int] = []


def interop_sks(n: int) -> list[int]:
    """sk_i for i < n (interop.ts:19-22), cached across calls."""
    while len(_SK_CACHE) < n:
        i = len(_SK_CACHE)
        _SK_CACHE.append(int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER)
    return _SK_CACHE[:n]


def message(j: int, tag: bytes = b"LODE") -> bytes:
    return hashlib.sha256(j.to_bytes(8, "little") + tag).digest()


def load_table(ctxs, n_keys: int) -> bytes:
    """Compressed pubkeys of interop keys 0..n_keys-1, loaded into every context's
    device table (made once on the first context).  Returns the 48-byte keys."""
    sks = interop_sks(n_keys)
    blob = b"".join(s.to_bytes(32, "big") for s in sks)
    pks = ctxs[0].sk_to_pk(blob).tobytes()
    for c in ctxs:
        codes = c.load_pubkeys(pks, 48)
        assert (codes == 0).all(), "interop pubkeys must decode"
    return pks


def _sign_all(gpu, sks: list[int], msgs: list[bytes]) -> list[bytes]:
    out = []
    step = 1 << 16
    for k in range(0, len(sks), step):
        blob = b"".join(s.to_bytes(32, "big") for s in sks[k:k + step])
        sig = gpu.sign(blob, b"".join(msgs[k:k + step]))
        out.extend(bytes(sig[i]) for i in range(sig.shape[0]))
    return out


@dataclass
class Workload:
    """Calls of sets (table index lists, 32-byte root, 96-byte signature), the
    validity of every set by construction, and how each call is submitted."""

    calls: list = field(default_factory=list)      # list[list[(idx_list, msg, sig)]]
    valid: list = field(default_factory=list)      # list[list[bool]], per call per set
    batchable: bool = False                        # one request per call (False) or one per set (True)
    note: str = ""

    @property
    def n_sets(self) -> int:
        return sum(len(c) for c in self.calls)

    def requests(self, k: int):
        """pack_requests input of call k: one non-batchable request, or one batchable
        request per set (gossip)."""
        sets = self.calls[k]
        return [(True, [s]) for s in sets] if self.batchable else [(False, list(sets))]

    def expected(self, k: int) -> list[bool]:
        """Per-request validity of call k (the verdict every correct verifier returns
        for an all-decodable call)."""
        v = self.valid[k]
        return list(v) if self.batchable else [all(v)]


def cfg3_block(gpu, n_keys: int, committee: int = 512, n_att: int = 128, seed: int = 1) -> Workload:
    rng = random.Random(seed)
    sks = interop_sks(n_keys)
    sets_idx = [rng.sample(range(n_keys), committee) for _ in range(n_att + 1)]  # + sync aggregate
    msgs = [message(j, b"CFG3") for j in range(n_att + 1)]
    agg_sks = [sum(sks[i] for i in idx) % R_ORDER for idx in sets_idx]
    sigs = _sign_all(gpu, agg_sks, msgs)
    sets = [(idx, m, s) for idx, m, s in zip(sets_idx, msgs, sigs)]
    return Workload(calls=[sets], valid=[[True] * len(sets)], batchable=False,
                    note=f"cfg3 block import: {n_att} aggregate sets x {committee} keys + 1 sync aggregate x "
                         f"{committee}, keys sampled without replacement from a {n_keys}-key table (seed {seed}), "
                         "one non-batchable request")


def cfg4_slice(gpu, n_keys: int, n_sets_total: int, rank: int = 0, world: int = 1, call_sets: int = 128,
               agg_frac: float = 0.10, agg_k: int = 128, invalid_frac: float = 0.01, seed: int = 2,
               batchable_calls: bool = False) -> Workload:
    """This GPU's calls of the cfg4 job: calls c with c % world == rank."""
    rng = random.Random(seed)
    sks = interop_sks(n_keys)
    n_calls = (n_sets_total + call_sets - 1) // call_sets
    mine = [c for c in range(n_calls) if c % world == rank]
    # every set's shape and fate is drawn from one stream, so every rank agrees
    plan = []
    for j in range(n_sets_total):
        is_agg = rng.random() < agg_frac
        idx = rng.sample(range(n_keys), agg_k) if is_agg else [rng.randrange(n_keys)]
        bad = rng.random() < invalid_frac
        kind = rng.randrange(2) if bad else -1
        plan.append((idx, kind))
    calls, valid, sign_sks, sign_msgs, slots = [], [], [], [], []
    for c in mine:
        sets, v = [], []
        for j in range(c * call_sets, min(n_sets_total, (c + 1) * call_sets)):
            idx, kind = plan[j]
            msg = message(j, b"CFG4")
            sk = sum(sks[i] for i in idx) % R_ORDER
            if kind == 0:    # signed over another message
                smsg = message(j + n_sets_total, b"CFG4")
            else:
                smsg = msg
            if kind == 1:    # signed by another key
                sk = (sk + 1) % R_ORDER
            sign_sks.append(sk)
            sign_msgs.append(smsg)
            slots.append((len(calls), len(sets)))
            sets.append([idx, msg, None])
            v.append(kind < 0)
        calls.append(sets)
        valid.append(v)
    for (ci, si), sig in zip(slots, _sign_all(gpu, sign_sks, sign_msgs)):
        calls[ci][si][2] = sig
    calls = [[tuple(s) for s in c] for c in calls]
    return Workload(calls=calls, valid=valid, batchable=batchable_calls,
                    note=f"cfg4 slice (rank {rank} of {world}): {sum(len(c) for c in calls)} of {n_sets_total} sets, "
                         f"{int(agg_frac * 100)} % aggregates of {agg_k} keys, {invalid_frac * 100:g} % invalid "
                         f"(seed {seed}), calls of {call_sets} sets"
                         + (", each set its own batchable request" if batchable_calls else
                            ", one non-batchable request per call"))


def cfg5_slice(gpu, n_keys: int, n_sets: int, n_roots: int, call_sets: int = 1024, invalid: int = 0,
               rank: int = 0, seed: int = 5) -> Workload:
    """n_sets single-pubkey attestations over n_roots committees of consecutive sets;
    `invalid` sets (uniform, seed) sign another root."""
    rng = random.Random(seed + rank)
    sks = interop_sks(n_keys)
    per_root = n_sets // n_roots
    roots = [message(rank * n_roots + k, b"CFG5") for k in range(n_roots)]
    keys = [rng.randrange(n_keys) for _ in range(n_sets)]
    bad = set(rng.sample(range(n_sets), invalid)) if invalid else set()
    msgs = [roots[min(j // per_root, n_roots - 1)] for j in range(n_sets)]
    smsgs = [message(10 ** 9 + j, b"CFG5") if j in bad else msgs[j] for j in range(n_sets)]
    sigs = _sign_all(gpu, [sks[k] for k in keys], smsgs)
    calls, valid = [], []
    for c in range(0, n_sets, call_sets):
        calls.append([([keys[j]], msgs[j], sigs[j]) for j in range(c, min(n_sets, c + call_sets))])
        valid.append([j not in bad for j in range(c, min(n_sets, c + call_sets))])
    return Workload(calls=calls, valid=valid, batchable=True,
                    note=f"cfg5 slice: {n_sets} single-pubkey attestations over {n_roots} committee roots "
                         f"({per_root} sets each), {invalid} invalid, calls of {call_sets} batchable single-set requests")


def packed_calls(w: Workload):
    from .native import pack_requests

    return [pack_requests(w.requests(k)) for k in range(len(w.calls))]


def verdicts_ok(w: Workload, k: int, v: np.ndarray) -> bool:
    return [int(x) for x in v] == [1 if e else 0 for e in w.expected(k)]
