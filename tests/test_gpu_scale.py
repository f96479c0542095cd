"""Parity at the per-GPU slices of BASELINE configs 4 and 5, on the GPU.

The sets are made on the device (lodestar_amd/workloads.py: interop keys in a 1M-key
device table, GPU signing, validity known by construction).  Expected per-request
verdicts and the worker's counters come from the oracle's worker semantics,
oracle.verify_many_signature_sets (multithread/worker.ts:32-108), run over tokens that
carry each set's outcome: `_token_maybe_batch` restates the oracle's
verify_signature_sets_maybe_batch rules (maybeBatch.ts:16-39) for sets whose
crypto outcome is known, so the chunking (chunkifyMaximizeChunkSize(reqs, 16)),
failing-chunk fallback, batchRetries and batchSigsSuccess the GPU reports are checked
against the oracle, not against rules re-derived in the test.

  cfg4: 125k sets (1M / 8 GPUs), 90 % single / 10 % aggregate of 128 keys, 1 % invalid
        (half over another message, half by another key), calls of 128 sets: once as
        range sync sends them (one non-batchable request per call) and once with every
        set its own batchable request (invalid sets fail the merged check and their
        chunks; the per-request fallback runs).
  cfg5: 131,072 single-pubkey attestations over 256 committee roots (2048 / 8) in calls
        of 1024 batchable requests, 64 of them invalid.
"""
from __future__ import annotations

import pytest

from lodestar_amd import workloads as W

pytestmark = pytest.mark.gpu

N_KEYS = 1 << 20


def _token_maybe_batch(oracle):
    """verify_signature_sets_maybe_batch (oracle) over outcome tokens: 1 valid, 0 invalid."""
    def maybe_batch(tokens):
        if len(tokens) == 0:
            raise oracle.BlsError(oracle.E_EMPTY_SET)
        return all(t == 1 for t in tokens)
    return maybe_batch


def _oracle_expect(oracle, w: W.Workload, calls):
    """Per call (one worker message each): (verdicts, batch_retries, batch_sigs_success)
    from oracle.verify_many_signature_sets over the calls' validity tokens."""
    mb = _token_maybe_batch(oracle)
    out = []
    for k in calls:
        v = w.valid[k]
        reqs = [(True, [1 if x else 0]) for x in v] if w.batchable else [(False, [1 if x else 0 for x in v])]
        res, retries, ok = oracle.verify_many_signature_sets(reqs, mb)
        verdicts = [(1 if r[1] else 0) if r[0] == "success" else -r[1].code for r in res]
        out.append((verdicts, retries, ok))
    return out


@pytest.fixture(scope="module")
def big():
    """A context holding the 1M-key interop table (96 MB of HBM)."""
    from lodestar_amd.native import GpuContext

    ctx = GpuContext(0)
    W.load_table([ctx], N_KEYS)
    yield ctx
    ctx.close()


def _check_workload(ctx, oracle, w: W.Workload, per_pass: int = 8):
    pbs = W.packed_calls(w)
    expect = _oracle_expect(oracle, w, range(len(pbs)))
    retries = ok = 0
    for g in range(0, len(pbs), per_pass):
        vs, st = ctx.verify_many(pbs[g:g + per_pass])
        for k, v in zip(range(g, g + per_pass), vs):
            assert [int(x) for x in v] == expect[k][0], f"call {k}"
        retries += st.batch_retries
        ok += st.batch_sigs_success
    assert retries == sum(e[1] for e in expect)
    assert ok == sum(e[2] for e in expect)
    return expect


@pytest.mark.parametrize("batchable", [False, True], ids=["range_sync_calls", "per_set_requests"])
def test_cfg4_slice_parity(big, oracle, batchable):
    w = W.cfg4_slice(big, N_KEYS, 125_000, batchable_calls=batchable)
    assert w.n_sets == 125_000 and len(w.calls) == 977
    n_inv = sum(not x for v in w.valid for x in v)
    assert 1000 <= n_inv <= 1500  # ~1 %
    expect = _check_workload(big, oracle, w)
    false_calls = sum(1 for e in expect if 0 in e[0])
    assert false_calls > 500  # ~72 % of 128-set calls hold an invalid set: the fallback path runs


def test_cfg5_slice_parity(big, oracle):
    w = W.cfg5_slice(big, N_KEYS, 131_072, 256, invalid=64)
    assert len(w.calls) == 128 and w.n_sets == 131_072
    expect = _check_workload(big, oracle, w)
    assert sum(e[0].count(0) for e in expect) == 64
    assert sum(e[1] for e in expect) > 0
