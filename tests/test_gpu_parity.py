"""GPU parity tests: every entry point of the C-ABI on cuda:0 against the golden
fixtures (tests/golden/golden.json, produced by the CPU oracle and pinned by the
reference's own known-answer data) and the reference's verdict semantics.

Bar: bit-exact for every byte output (hash_to_G2, aggregate pubkeys, pk, signatures);
exact verdict / error-code equality for verification.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from lodestar_amd._abi import (
    CODE_BAD_ENCODING,
    CODE_EMPTY_AGGREGATE,
    CODE_EMPTY_SET,
    CODE_INVALID_SIZE,
    CODE_PK_IS_INFINITY,
    CODE_POINT_NOT_IN_GROUP,
    CODE_POINT_NOT_ON_CURVE,
    CODE_ZERO_SIGNATURE,
)
from lodestar_amd.native import pack_requests

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module", params=["pset", "sigagg"])
def verify_path(request, gpu):
    """Every test of this module runs on both per-set paths: the all-cooperative k_pset
    and the aggregated-signature path (k_chain + k_gsum / k_vset + single-pair k_mln),
    whatever the call size would pick."""
    from lodestar_amd._abi import DEBUG_MERGED_EVERY_PASS, DEBUG_SIGAGG_OFF, DEBUG_SIGAGG_ON

    # the merged check on every pass (a test's merged_check expectation must not depend on
    # what the previous test left on the shared context); the adaptive skip after a failed
    # pass is test_merged_check_skipped_after_failing_pass below
    gpu.base_debug_flags = (DEBUG_SIGAGG_ON if request.param == "sigagg" else DEBUG_SIGAGG_OFF) | \
        DEBUG_MERGED_EVERY_PASS
    gpu.set_debug_flags(0)
    yield request.param
    gpu.base_debug_flags = 0
    gpu.set_debug_flags(0)


def _h(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def test_hash_to_g2_bit_exact(gpu, golden):
    vecs = golden["hash_to_g2"]
    msgs = b"".join(bytes.fromhex(v["msg"]) for v in vecs)
    out = gpu.hash_to_g2(msgs)
    for row, v in zip(out, vecs):
        assert row.tobytes().hex() == v["point"]


def test_sk_to_pk_interop_kat(gpu, golden, oracle):
    sks = b"".join(oracle.interop_secret_key(i).to_bytes(32, "big") for i in range(100))
    pks = gpu.sk_to_pk(sks)
    assert [p.tobytes().hex() for p in pks] == golden["kat2_interop_pubkeys"]
    assert pks[0].tobytes().hex() == golden["kat1"]["pubkey"]


def test_sign_kat_and_golden(gpu, golden):
    k = golden["kat1"]
    sig = gpu.sign(bytes.fromhex(k["sk"]), bytes.fromhex(k["signing_root"]))
    assert sig[0].tobytes().hex() == k["signature"]
    sv = golden["signatures"]
    sks = b"".join(bytes.fromhex(s["sk"]) for s in sv)
    msgs = b"".join(bytes.fromhex(s["msg"]) for s in sv)
    out = gpu.sign(sks, msgs)
    assert [o.tobytes().hex() for o in out] == [s["sig"] for s in sv]


@pytest.fixture(scope="module")
def table(gpu, golden):
    """Device pubkey table: the 100 interop keys (KAT-2), compressed, loaded once."""
    pks = b"".join(bytes.fromhex(h) for h in golden["kat2_interop_pubkeys"])
    base = gpu.load_pubkeys(b"", 48)  # current size probe
    codes = gpu.load_pubkeys(pks, 48)
    assert (codes == 0).all()
    return 0 if base.size == 0 else None


def test_aggregate_pubkeys_bit_exact(gpu, golden, table):
    agg = golden["aggregate"]
    out, codes = gpu.aggregate_pubkeys(agg["lists"])
    assert list(codes) == [0] * len(agg["lists"])
    assert [o.hex() for o in out] == agg["expected"]
    _, codes = gpu.aggregate_pubkeys([[]])
    assert codes[0] == CODE_EMPTY_AGGREGATE


# ---------------------------------------------------------------------------
# verification semantics (worker.ts:32-108, maybeBatch.ts:16-39, multithread.test.ts)
# ---------------------------------------------------------------------------
def _keys(oracle, n):
    return [oracle.interop_secret_key(i).to_bytes(32, "big") for i in range(n)]


def _sets(gpu, oracle, n, tag=b"m"):
    sks = _keys(oracle, n)
    msgs = [_h(tag + b"%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks), b"".join(msgs))
    return [([i], msgs[i], sigs[i].tobytes()) for i in range(n)]


def test_verify_valid_single_and_batched(gpu, oracle, table):
    sets = _sets(gpu, oracle, 3)
    # 1 request of 3 sets (non-batchable), 8 copies batchable (multithread.test.ts:52-87)
    reqs = [(False, sets)] + [(True, sets)] * 8 + [(False, sets[:1])]
    v, st = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == [1] * 10
    assert st.batch_retries == 0 and st.batch_sigs_success == 24


def test_verify_invalid_size_isolated(gpu, oracle, table):
    # multithread.test.ts:89-106: a 32-byte signature rejects with BLST_INVALID_SIZE,
    # 8 concurrent valid requests still resolve true
    sets = _sets(gpu, oracle, 3)
    bad = [(sets[0][0], sets[0][1], bytes(32))]
    reqs = [(True, bad)] + [(True, sets)] * 8
    v, st = gpu.verify_packed(pack_requests(reqs))
    assert v[0] == -CODE_INVALID_SIZE
    assert list(v[1:]) == [1] * 8
    assert st.batch_retries == 0 or st.batch_retries == st.n_chunks


def test_verify_wrong_message_and_key(gpu, oracle, table):
    sets = _sets(gpu, oracle, 4)
    wrong_msg = [(sets[0][0], _h(b"other"), sets[0][2])]
    wrong_key = [([1], sets[0][1], sets[0][2])]
    reqs = [(False, wrong_msg), (False, wrong_key), (False, sets), (False, sets[:3] + wrong_msg)]
    v, _ = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == [0, 0, 1, 0]
    # the same requests batchable: the batch fails and the fallback isolates them
    v2, st = gpu.verify_packed(pack_requests([(True, r[1]) for r in reqs]))
    assert list(v2) == [0, 0, 1, 0]
    assert st.batch_retries >= 1


def test_verify_decode_error_codes(gpu, oracle, golden, table):
    sets = _sets(gpu, oracle, 2)
    reqs, expect = [], []
    for case in golden["sig_decode"]:
        raw = bytes.fromhex(case["bytes"])
        reqs.append((False, [(sets[0][0], sets[0][1], raw)]))
        if case["code"] != 0:
            expect.append(-case["code"])
        elif case["name"] == "infinity":
            expect.append(-CODE_ZERO_SIGNATURE)  # 1-set path rejects the infinity signature
        else:
            expect.append(0)  # a valid G2 point, but not the signature of this message
    v, _ = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == expect


def test_verify_edge_cases(gpu, oracle, table):
    sets = _sets(gpu, oracle, 3)
    inf_sig = bytes([0xC0]) + bytes(95)
    reqs = [
        (False, []),                                       # empty -> "Empty signature set"
        (False, [sets[0], (sets[1][0], sets[1][1], inf_sig)]),  # n >= 2 with an infinity sig -> false
        (False, [([], sets[0][1], sets[0][2])]),           # empty aggregate
        (False, [([0, 1], sets[0][1], sets[0][2])]),       # aggregate of 2 keys, sig of key 0 -> false
        (True, sets),
    ]
    v, _ = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == [-CODE_EMPTY_SET, 0, -CODE_EMPTY_AGGREGATE, 0, 1]


def test_large_groups_multi_level_sums(gpu, oracle, table):
    """Requests of many sets: one batchable request of 300 sets (its chunk's r sig sum
    runs several k_gsum levels), non-batchable requests of 70 and 2 sets (individual
    groups summed in the individual pass), one of them with an invalid set; verdicts
    with the merged check on and off."""
    from lodestar_amd._abi import DEBUG_NO_MERGED_CHECK

    n = 300
    sks = _keys(oracle, 100)
    msgs = [_h(b"big-%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 100] for i in range(n)), b"".join(msgs))
    sets = [([i % 100], msgs[i], sigs[i].tobytes()) for i in range(n)]
    bad70 = list(sets[100:170])
    bad70[37] = (bad70[37][0], _h(b"tampered"), bad70[37][2])
    reqs = [(True, sets), (False, sets[:70]), (False, bad70), (False, sets[200:202]), (True, sets[250:300])]
    for flags in (0, DEBUG_NO_MERGED_CHECK):
        try:
            gpu.set_debug_flags(flags)
            v, st = gpu.verify_packed(pack_requests(reqs))
        finally:
            gpu.set_debug_flags(0)
        assert list(v) == [1, 1, 0, 1, 1], flags
        assert st.n_individual == 3
    # the same with the big request invalid: its chunk fails, it is retried on its own
    bad = list(sets)
    bad[299] = (bad[299][0], bad[299][1], sets[0][2])
    v, st = gpu.verify_packed(pack_requests([(True, bad), (True, sets[250:300])]))
    assert list(v) == [0, 1] and st.batch_retries == 1 and st.n_individual == 2


def test_verify_aggregate_sets(gpu, oracle, table):
    # fast-aggregate style sets: the same message signed by k keys, aggregated G2 signature
    k = 5
    msg = _h(b"committee")
    sks = _keys(oracle, k)
    sigs = gpu.sign(b"".join(sks), msg * k)
    pts = [oracle.signature_from_bytes(s.tobytes()) for s in sigs]
    agg = None
    for p_ in pts:
        agg = oracle.E2.add(agg, p_)
    agg_sig = oracle.g2_compress(agg)
    reqs = [(False, [(list(range(k)), msg, agg_sig)]), (False, [(list(range(k - 1)), msg, agg_sig)])]
    v, _ = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == [1, 0]


def test_verify_raw_pubkeys(gpu, oracle, golden):
    # raw 96-byte uncompressed keys (what index.ts:160 sends the worker)
    sks = _keys(oracle, 3)
    msgs = [_h(b"raw%d" % i) for i in range(3)]
    sigs = gpu.sign(b"".join(sks), b"".join(msgs))
    raw = [oracle.g1_serialize(oracle.sk_to_pk(int.from_bytes(s, "big"))) for s in sks]
    sets = [(raw[i], msgs[i], sigs[i].tobytes()) for i in range(3)]
    reqs = [(False, sets), (True, sets[:1]), (True, sets[1:])]
    v, _ = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == [1, 1, 1]
    # deserializeSet maps every request of the worker message before verifying and
    # throws on the first undecodable key (worker.ts:43-46); the pool then rejects
    # every job of that message (index.ts:367-374): all four requests reject.
    bad_pk = bytes([0x80]) + raw[0][1:]          # compression flag on a 96-byte key
    off_curve = raw[1][:48] + raw[2][48:]         # (x1, y2): not on the curve
    for bad, code in ((bad_pk, CODE_BAD_ENCODING), (off_curve, CODE_POINT_NOT_ON_CURVE)):
        reqs = [(False, sets), (True, sets[:1]), (True, sets[1:]), (False, [(bad, msgs[0], sigs[0].tobytes())])]
        v, _ = gpu.verify_packed(pack_requests(reqs))
        assert list(v) == [-code] * 4
        want, _, _ = oracle.verify_many_signature_sets(reqs)
        assert [-r[1].code for r in want] == list(v)
    # two bad keys: the first in request order names the error
    reqs = [(True, sets[:1]), (True, [(off_curve, msgs[0], sigs[0].tobytes())]),
            (True, [(bad_pk, msgs[0], sigs[0].tobytes())])]
    v, _ = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == [-CODE_POINT_NOT_ON_CURVE] * 3


def test_verify_batch_with_injected_invalid(gpu, oracle, table):
    """64 single-set batchable requests, 3 invalid: chunks of 16 requests; the chunks
    holding an invalid set fail and are re-verified per request."""
    n = 64
    sks = _keys(oracle, 16)
    msgs = [_h(b"batch%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))
    bad = {5, 17, 40}
    reqs = []
    for i in range(n):
        m = msgs[i] if i not in bad else _h(b"tampered%d" % i)
        reqs.append((True, [([i % 16], m, sigs[i].tobytes())]))
    v, st = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == [0 if i in bad else 1 for i in range(n)]
    assert st.n_chunks == 4 and st.batch_retries == 3
    assert st.batch_sigs_success == 16


def test_verify_pk_infinity(gpu, oracle):
    inf_pk = bytes([0x40]) + bytes(95)
    sets = [(inf_pk, _h(b"x"), bytes.fromhex("c0" + "00" * 95))]
    v, _ = gpu.verify_packed(pack_requests([(False, sets)]))
    assert v[0] == -CODE_ZERO_SIGNATURE
    sk = _keys(oracle, 1)[0]
    sig = gpu.sign(sk, _h(b"x"))[0].tobytes()
    v, _ = gpu.verify_packed(pack_requests([(False, [(inf_pk, _h(b"x"), sig)])]))
    assert v[0] == -CODE_PK_IS_INFINITY


def test_fp_mul_device_vs_bigint(gpu):
    """The device Montgomery product (inline-asm product scanning on gfx950) against
    Python big integers: random operands plus the edges 0, 1, p-1, 2^381 region."""
    import random

    from oracle.bls_oracle import P

    rng = random.Random(7)
    vals = [0, 1, 2, P - 1, P - 2, (1 << 380), (1 << 381) % P, P // 2, P // 2 + 1]
    a = vals + [rng.randrange(P) for _ in range(500)]
    b = list(reversed(vals)) + [rng.randrange(P) for _ in range(500)]
    sq = vals + [rng.randrange(P) for _ in range(200)]      # squares: the dedicated fp_sqr
    a, b = a + sq, b + sq
    out = gpu.fp_mul_test(b"".join(x.to_bytes(48, "big") for x in a), b"".join(x.to_bytes(48, "big") for x in b))
    got = [int.from_bytes(out[48 * i: 48 * i + 48], "big") for i in range(len(a))]
    assert got == [(x * y) % P for x, y in zip(a, b)]


@pytest.mark.gpu
def test_exact_path_matches_cooperative_path(gpu, oracle, golden, table):
    """The same calls with every set forced through the exact path (complete single-lane
    formulas) give the verdicts of the cooperative k_pset path."""
    sets = _sets(gpu, oracle, 4, tag=b"exact")
    reqs = [(True, [s]) for s in sets] + [(False, sets)]
    reqs.append((True, [(sets[0][0], _h(b"other"), sets[0][2])]))          # wrong message
    for case in golden["sig_decode"]:                                       # decode / subgroup codes
        reqs.append((False, [(sets[0][0], sets[0][1], bytes.fromhex(case["bytes"]))]))
    pb = pack_requests(reqs)
    v0, st0 = gpu.verify_packed(pb)
    try:
        gpu.set_debug_flags(1)
        v1, st1 = gpu.verify_packed(pb)
    finally:
        gpu.set_debug_flags(0)
    assert list(v0) == list(v1)
    assert st1.n_flagged >= 5 and st0.n_flagged < st1.n_flagged
    assert list(v0[:5]) == [1] * 5 and v0[5] == 0


@pytest.mark.gpu
def test_merged_check_matches_chunk_verdicts(gpu, oracle, table):
    """The merged check (one final exponentiation over all chunks' sets) passes only
    when every chunk would; otherwise the per-chunk verdicts decide, so verdicts and
    stats equal those of the chunked worker (worker.ts:56-88) with it switched off."""
    from lodestar_amd._abi import DEBUG_NO_MERGED_CHECK

    n = 48
    sks = _keys(oracle, 16)
    msgs = [_h(b"merged%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))
    good = [(True, [([i % 16], msgs[i], sigs[i].tobytes())]) for i in range(n)]
    one_bad = list(good)
    one_bad[20] = (True, [([20 % 16], _h(b"tampered"), sigs[20].tobytes())])
    err = list(good)
    err[33] = (True, [([33 % 16], msgs[33], bytes(32))])  # BLST_INVALID_SIZE inside a chunk
    for reqs, merged_expect in ((good, 1), (one_bad, 2), (err, 2)):
        pb = pack_requests(reqs)
        v0, st0 = gpu.verify_packed(pb)
        try:
            gpu.set_debug_flags(DEBUG_NO_MERGED_CHECK)
            v1, st1 = gpu.verify_packed(pb)
        finally:
            gpu.set_debug_flags(0)
        assert list(v0) == list(v1)
        assert st0.merged_check == merged_expect and st1.merged_check == 0
        assert (st0.batch_retries, st0.batch_sigs_success, st0.n_chunks) == \
            (st1.batch_retries, st1.batch_sigs_success, st1.n_chunks)
    assert list(v0) == [1] * 33 + [-CODE_INVALID_SIZE] + [1] * 14


@pytest.mark.gpu
def test_committee_shared_roots_dedup(gpu, oracle, table):
    """gossip attestations of one committee share a
    signing root, so hash_to_field + SSWU run once per distinct root (n_unique_msgs).
    Verdicts match the per-set pre-stage and the exact path, with invalid sets (a
    signature over another root, a wrong key) mixed into the shared-root chunks."""
    from lodestar_amd._abi import DEBUG_FORCE_EXACT, DEBUG_NO_MSG_DEDUP

    n = 48
    roots = [_h(b"committee-root%d" % k) for k in range(3)]
    sks = _keys(oracle, 16)
    msgs = [roots[(i * 7) % 3] for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))
    reqs, expect = [], []
    for i in range(n):
        sig, pk = sigs[i].tobytes(), [i % 16]
        if i == 9:
            sig = sigs[10].tobytes() if msgs[10] != msgs[9] else sigs[11].tobytes()  # other root
        if i == 30:
            pk = [(i + 1) % 16]  # another committee member's key
        reqs.append((True, [(pk, msgs[i], sig)]))
        expect.append(0 if i in (9, 30) else 1)
    reqs.append((False, [([i % 16], msgs[i], sigs[i].tobytes()) for i in range(12)]))  # 1 request, 12 sets, 3 roots
    expect.append(1)
    pb = pack_requests(reqs)
    v0, st0 = gpu.verify_packed(pb)
    assert list(v0) == expect
    assert st0.n_unique_msgs == 3
    results = {}
    for flags in (DEBUG_NO_MSG_DEDUP, DEBUG_FORCE_EXACT):
        try:
            gpu.set_debug_flags(flags)
            results[flags] = gpu.verify_packed(pb)
        finally:
            gpu.set_debug_flags(0)
    assert list(results[DEBUG_NO_MSG_DEDUP][0]) == expect
    assert results[DEBUG_NO_MSG_DEDUP][1].n_unique_msgs == n + 12
    assert list(results[DEBUG_FORCE_EXACT][0]) == expect


# ---------------------------------------------------------------------------
# one call sharded into Fp12 partials + one final exponentiation
# ---------------------------------------------------------------------------
def test_sharded_partials_final_check(gpu, oracle, table):
    from lodestar_amd.shard import shard_bounds

    seed = bytes(range(32))
    sets = _sets(gpu, oracle, 10, tag=b"shard")
    bounds = shard_bounds(len(sets), 3)

    def partials(ss):
        out = []
        for beg, end in bounds:
            p, st, _, _ = gpu.partial(pack_requests([(True, ss[beg:end])], seed=seed), beg)
            assert st == 0
            out.append(p)
        return out

    good = partials(sets)
    assert gpu.final_check(good)
    assert gpu.final_check(good[::-1])                    # the product is order-free
    # the same call verified unsharded agrees
    v, _ = gpu.verify_packed(pack_requests([(False, sets)], seed=seed))
    assert v[0] == 1
    # one invalid set (wrong message) in the last shard: the call fails, its shard is found
    bad = list(sets)
    bad[8] = (bad[8][0], _h(b"tampered"), bad[8][2])
    ps = partials(bad)
    assert not gpu.final_check(ps)
    assert [gpu.final_check([p]) for p in ps] == [True, True, False]
    # an undecodable signature rejects the call with its code
    enc = list(sets)
    enc[4] = (enc[4][0], enc[4][1], b"\x00" * 96)
    beg, end = bounds[1]
    p, st, err, _ = gpu.partial(pack_requests([(True, enc[beg:end])], seed=seed), beg)
    assert p is None and st == -CODE_BAD_ENCODING and err == (1, 4 - beg)


def _sharded_gpu_rank(rank, world, port, sets, q, flags=0):
    import os

    import torch.distributed as dist

    from lodestar_amd.native import GpuContext
    from lodestar_amd.shard import GpuPartialBackend, verify_call_sharded

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    with GpuContext(0) as gpu:
        gpu.set_debug_flags(flags)  # the parent's per-set path (the module's verify_path)
        be = GpuPartialBackend(gpu)
        for ss in sets:
            out.append(verify_call_sharded(ss, bytes(32), be, dist))
    q.put((rank, out))
    dist.destroy_process_group()


def test_sharded_call_two_ranks(gpu, oracle):
    """Two processes (gloo exchange of the 580-byte records; both ranks on cuda:0)."""
    import socket

    import torch.multiprocessing as mp

    sks = _keys(oracle, 6)
    msgs = [_h(b"r2-%d" % i) for i in range(6)]
    sigs = gpu.sign(b"".join(sks), b"".join(msgs))
    raw = [oracle.g1_serialize(oracle.sk_to_pk(int.from_bytes(s, "big"))) for s in sks]
    good = [(raw[i], msgs[i], sigs[i].tobytes()) for i in range(6)]
    bad = good[:1] + [(raw[1], msgs[2], sigs[1].tobytes())] + good[2:]
    two_inf = [good[0], (raw[1], msgs[1], bytes([0xC0]) + bytes(95))]
    order = [(raw[0], msgs[0], bytes(32))] + good[1:5] + [(bytes([0x80]) + raw[5][1:], msgs[5], sigs[5].tobytes())]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_gpu_rank, args=(r, 2, port, [good, bad, two_inf, order], q,
                                                        gpu.base_debug_flags)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in (0, 1):
        assert res[r][0] == (True, {"bad_shards": []})
        assert res[r][1] == (False, {"bad_shards": [0]})
        assert res[r][2] == (False, {"bad_shards": []}) or res[r][2][0] is False   # infinity sig, 1-set shards
        assert res[r][3][0] == -CODE_BAD_ENCODING                                  # pubkey error beats signature


def test_sharded_call_two_ranks_large(gpu, oracle):
    """The sharded call at the per-GPU scale of a pass: 2,048 sets over two processes
    (1,024 per rank), all valid, then one set signing another message in rank 1's shard:
    the call fails and only shard 1 is reported bad.  Each rank's partial runs on the
    module's path (the verify_path fixture's debug flag is handed to the children: a
    1,024-set shard would otherwise take the per-set path whenever few sets are in
    flight, bls_gpu.hip use_sigagg), so the aggregated sharded path is covered at pass
    scale too."""
    import socket

    import torch.multiprocessing as mp

    n = 2048
    sks = _keys(oracle, 16)
    msgs = [_h(b"r2big-%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))
    raw = [oracle.g1_serialize(oracle.sk_to_pk(int.from_bytes(s, "big"))) for s in sks]
    good = [(raw[i % 16], msgs[i], sigs[i].tobytes()) for i in range(n)]
    bad = list(good)
    bad[1500] = (raw[1500 % 16], msgs[7], sigs[1500].tobytes())
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_gpu_rank, args=(r, 2, port, [good, bad], q, gpu.base_debug_flags))
             for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=110) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in (0, 1):
        assert res[r][0] == (True, {"bad_shards": []})
        assert res[r][1] == (False, {"bad_shards": [1]})


# ---------------------------------------------------------------------------
# BASELINE configs as parity cases (size-independent properties)
# ---------------------------------------------------------------------------
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _interop_sks(n):
    return [int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER for i in range(n)]


@pytest.fixture(scope="module")
def big_table():
    """A separate context with a 65,536-key device table (interop keys), so the
    session's `gpu` table stays as the other tests expect."""
    from lodestar_amd.native import GpuContext

    n = 65536
    sks = _interop_sks(n)
    ctx = GpuContext(0)
    pks = ctx.sk_to_pk(b"".join(s.to_bytes(32, "big") for s in sks))
    assert (ctx.load_pubkeys(pks.tobytes(), 48) == 0).all()
    yield ctx, sks, pks
    ctx.close()


def test_cfg3_block_import_aggregates(big_table, oracle):
    """cfg3: one block = 128 aggregate sets x 512 distinct pubkeys + the sync aggregate
    x 512 (indices sampled without replacement; table of 65,536 keys instead of 1M),
    verified as one call.  Aggregate signatures are made with the summed secret key
    (sum_j sk_j H(m) = sum_j sig_j).  Valid -> true; one tampered set -> false; the
    device aggregate pubkeys equal the oracle's for two sets."""
    ctx, sks, _ = big_table
    rng = np.random.default_rng(1)
    n_sets, k = 129, 512
    idx = [sorted(rng.choice(len(sks), size=k, replace=False).tolist()) for _ in range(n_sets)]
    msgs = [_h(b"block%d" % i) for i in range(n_sets)]
    agg_sks = [sum(sks[j] for j in ix) % R_ORDER for ix in idx]
    sigs = ctx.sign(b"".join(s.to_bytes(32, "big") for s in agg_sks), b"".join(msgs))
    sets = [(idx[i], msgs[i], sigs[i].tobytes()) for i in range(n_sets)]
    v, _ = ctx.verify_packed(pack_requests([(False, sets)]))
    assert v[0] == 1
    bad = list(sets)
    bad[77] = (idx[77][:-1], msgs[77], sigs[77].tobytes())       # one signer missing
    v, _ = ctx.verify_packed(pack_requests([(False, bad), (True, sets[:64]), (True, sets[64:])]))
    assert list(v) == [0, 1, 1]
    outs, codes = ctx.aggregate_pubkeys([idx[0], idx[128]])
    assert list(codes) == [0, 0]
    for o, ix in zip(outs, (idx[0], idx[128])):
        assert o == oracle.g1_serialize(oracle.sk_to_pk(sum(sks[j] for j in ix) % R_ORDER))


def test_cfg4_range_sync_mixed_with_invalid(big_table):
    """cfg4 at 1/64 scale on one GPU: 16,384 sets, 90% single / 10% aggregate (k=128),
    1% invalid (half wrong message, half another key's signature, seed 2), grouped
    into calls of 128 sets; each call's verdict equals the expected one."""
    ctx, sks, _ = big_table
    rng = np.random.default_rng(2)
    n = 16384
    is_agg = rng.random(n) < 0.10
    idx = [sorted(rng.choice(len(sks), size=128, replace=False).tolist()) if a else [int(rng.integers(len(sks)))]
           for a in is_agg]
    msgs = [_h(b"range%d" % i) for i in range(n)]
    sk_of = [sum(sks[j] for j in ix) % R_ORDER for ix in idx]
    bad = set(rng.choice(n, size=n // 100, replace=False).tolist())
    wrong_key = {i for i in bad if rng.random() < 0.5}
    sign_sk = [sk_of[(i + 1) % n] if i in wrong_key else sk_of[i] for i in range(n)]
    sigs = ctx.sign(b"".join(s.to_bytes(32, "big") for s in sign_sk), b"".join(msgs))
    sets = []
    for i in range(n):
        m = _h(b"wrong%d" % i) if (i in bad and i not in wrong_key) else msgs[i]
        sets.append((idx[i], m, sigs[i].tobytes()))
    calls = [sets[c:c + 128] for c in range(0, n, 128)]
    v, st = ctx.verify_packed(pack_requests([(False, c) for c in calls]))
    expect = [0 if any(i in bad for i in range(c, c + 128)) else 1 for c in range(0, n, 128)]
    assert list(v) == expect
    assert 0 < sum(expect) < len(expect)


def test_validate_pubkeys_matches_oracle(gpu, oracle, golden):
    """bls_gpu_validate_pubkeys (Scott's G1 test) vs the oracle's r*P == O KeyValidate:
    KAT-2 keys, infinity, on-curve points outside G1, bad encodings; 48- and 96-byte forms."""
    keys = [bytes.fromhex(h) for h in golden["kat2_interop_pubkeys"][:20]]
    x, outside = 1, []
    while len(outside) < 6:
        y = oracle.fp_sqrt((x ** 3 + 4) % oracle.P)
        if y is not None and not oracle.g1_in_subgroup((x, y)):
            outside.append((x, y))
        x += 1
    keys += [oracle.g1_compress(p_) for p_ in outside]
    keys += [bytes([0xC0]) + bytes(47), bytes(48), bytes([0xFF]) * 48]
    expect = [oracle.key_validate(k) for k in keys]
    assert list(gpu.validate_pubkeys(b"".join(keys), 48)) == expect
    raw = [oracle.g1_serialize(oracle.g1_decompress(k)[1]) for k in keys[:26]]
    assert list(gpu.validate_pubkeys(b"".join(raw), 96)) == expect[:26]


# ---------------------------------------------------------------------------
# The headline call (cfg2) and the epoch shape (cfg5) at full size, with invalid sets
# in every position that matters: chunk boundaries (chunks of 16 requests,
# worker.ts:17,56) and every slot of a packed wavefront (1, 2 or 3 sets per
# wavefront, kernels/k_pset.hip), through every packing, the merged check on / off
# and the exact path.  Reference: worker.ts:54-98, multithread.test.ts:89-106.
# ---------------------------------------------------------------------------
def _decode_case(golden, name):
    return bytes.fromhex(next(c["bytes"] for c in golden["sig_decode"] if c["name"] == name))


def _expected_stats(oracle, expect):
    """batch_retries / batch_sigs_success of one worker message of single-set batchable
    requests, from the oracle's worker semantics (oracle.verify_many_signature_sets,
    worker.ts:32-108) over outcome tokens: each set is its known outcome (1 valid, 0
    invalid, -code).  The token predicate restates oracle.verify_signature_sets_maybe_batch
    (maybeBatch.ts:16-39): every signature is decoded first and a decode error throws;
    one set alone verifies deterministically (an infinity signature throws
    ZERO_SIGNATURE there, and only makes a batch false); otherwise the batch is valid iff
    every set is.  The oracle's per-request verdicts must equal `expect`."""
    zero = -oracle.E_ZERO_SIGNATURE

    def maybe_batch(tokens):
        if len(tokens) == 0:
            raise oracle.BlsError(oracle.E_EMPTY_SET)
        for t in tokens:
            if t < 0 and t != zero:
                raise oracle.BlsError(-t)
        if len(tokens) == 1 and tokens[0] == zero:
            raise oracle.BlsError(oracle.E_ZERO_SIGNATURE)
        return all(t == 1 for t in tokens)

    res, retries, ok = oracle.verify_many_signature_sets([(True, [c]) for c in expect], maybe_batch)
    assert [(1 if r[1] else 0) if r[0] == "success" else -r[1].code for r in res] == list(expect)
    return retries, ok


def _run_all_paths(gpu, pb):
    """(verdicts, stats) of one call through: packings 1/2/3 (merged check on), the
    packing chosen by size with the merged check off, and the exact path."""
    from lodestar_amd._abi import DEBUG_FORCE_EXACT, DEBUG_NO_MERGED_CHECK, DEBUG_PACK

    out = {}
    for name, flags in (("auto", 0), ("pack1", DEBUG_PACK(1)), ("pack2", DEBUG_PACK(2)), ("pack3", DEBUG_PACK(3)),
                        ("no_merged", DEBUG_NO_MERGED_CHECK), ("exact", DEBUG_FORCE_EXACT)):
        try:
            gpu.set_debug_flags(flags)
            out[name] = gpu.verify_packed(pb)
        finally:
            gpu.set_debug_flags(0)
    return out


def test_cfg2_1024_call_with_invalid_sets(gpu, oracle, golden, table):
    """cfg2: 1024 single-set batchable requests in one call (64 chunks of 16).  Invalid
    sets straddle chunk boundaries and sit in every wavefront slot: wrong message, wrong
    key, a 32-byte signature, an on-curve point outside G2, the infinity signature,
    undecodable bytes.  Every path gives the reference verdicts and worker stats."""
    n = 1024
    sks = _keys(oracle, 100)
    msgs = [_h(b"cfg2-%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 100] for i in range(n)), b"".join(msgs))
    sets = [([i % 100], msgs[i], sigs[i].tobytes()) for i in range(n)]
    inf_sig = bytes([0xC0]) + bytes(95)
    bad = {
        15: ("msg", 0), 16: ("key", 0), 17: ("size", -CODE_INVALID_SIZE),            # chunk 0 / 1 boundary
        31: ("group", -CODE_POINT_NOT_IN_GROUP), 32: ("inf", -CODE_ZERO_SIGNATURE),  # chunk 1 / 2
        100: ("msg", 0), 101: ("msg", 0), 102: ("key", 0),                           # slots 1,2,0 of 3-packs
        511: ("curve", -CODE_POINT_NOT_ON_CURVE), 512: ("enc", -CODE_BAD_ENCODING),  # mid-call boundary
        700: ("inf", -CODE_ZERO_SIGNATURE), 701: ("group", -CODE_POINT_NOT_IN_GROUP),
        1021: ("key", 0), 1022: ("size", -CODE_INVALID_SIZE), 1023: ("msg", 0),      # last chunk, last slots
    }
    reqs, expect = [], []
    for i, (pk, m, sig) in enumerate(sets):
        kind, code = bad.get(i, (None, 1))
        if kind == "msg":
            m = _h(b"tampered%d" % i)
        elif kind == "key":
            pk = [(i + 1) % 100]
        elif kind == "size":
            sig = sig[:32]
        elif kind == "group":
            sig = _decode_case(golden, "not_in_group")
        elif kind == "curve":
            sig = _decode_case(golden, "not_on_curve")
        elif kind == "enc":
            sig = _decode_case(golden, "x_ge_p")
        elif kind == "inf":
            sig = inf_sig
        reqs.append((True, [(pk, m, sig)]))
        expect.append(code)
    pb = pack_requests(reqs)
    retries, ok = _expected_stats(oracle, expect)
    res = _run_all_paths(gpu, pb)
    for name, (v, st) in res.items():
        assert list(v) == expect, name
        assert (st.n_chunks, st.batch_retries, st.batch_sigs_success) == (64, retries, ok), name
    assert res["auto"][1].merged_check == 2 and res["no_merged"][1].merged_check == 0
    # every set that decodes goes through the exact path (the 4 decode failures never reach it)
    assert res["exact"][1].n_flagged == n - 4
    # the same call all-valid: the merged check passes on every packing
    good = pack_requests([(True, [s]) for s in sets])
    for name, (v, st) in _run_all_paths(gpu, good).items():
        assert list(v) == [1] * n, name
        assert st.batch_retries == 0 and st.batch_sigs_success == n, name
        assert st.merged_check == (0 if name == "no_merged" else 1), name


def test_cfg5_shape_two_roots_with_invalid(gpu, oracle, table, verify_path):
    """cfg5 shape: 1024 attestations of two committees sharing two signing
    roots, with invalid sets (a signature over the other root, a wrong key, an
    undecodable signature) in both committees; verdicts equal with root dedup on / off,
    every packing and the exact path."""
    from lodestar_amd._abi import DEBUG_NO_MSG_DEDUP, DEBUG_NO_UNITS

    n = 1024
    roots = [_h(b"epoch-root-a"), _h(b"epoch-root-b")]
    sks = _keys(oracle, 100)
    msgs = [roots[i * 2 // n] for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 100] for i in range(n)), b"".join(msgs))
    reqs, expect = [], []
    for i in range(n):
        pk, sig, code = [i % 100], sigs[i].tobytes(), 1
        if i in (3, 600):            # signature over the other committee's root
            sig, code = sigs[n - 1 - i].tobytes(), 0
        if i in (257, 1000):         # another validator's key
            pk, code = [(i + 7) % 100], 0
        if i in (0, 513):            # undecodable; set 0 is its root's first set, the one
            sig, code = bytes(96), -CODE_BAD_ENCODING  # that computes the shared H(m)
        reqs.append((True, [(pk, msgs[i], sig)]))
        expect.append(code)
    pb = pack_requests(reqs)
    res = _run_all_paths(gpu, pb)
    for name, flags in (("no_dedup", DEBUG_NO_MSG_DEDUP), ("no_units", DEBUG_NO_UNITS)):
        try:
            gpu.set_debug_flags(flags)
            res[name] = gpu.verify_packed(pb)
        finally:
            gpu.set_debug_flags(0)
    retries, ok = _expected_stats(oracle, expect)
    for name, (v, st) in res.items():
        assert list(v) == expect, name
        assert (st.batch_retries, st.batch_sigs_success) == (retries, ok), name
    assert res["auto"][1].n_unique_msgs == 2 and res["no_dedup"][1].n_unique_msgs == n
    # aggregated-signature path: one Miller loop per (chunk, root) -- 64 chunks of 16
    # requests, the roots change at a chunk boundary (set 512)
    assert res["auto"][1].n_ml_units == (64 if verify_path == "sigagg" else 0)
    assert res["no_units"][1].n_ml_units == 0
    # all valid: the merged check passes over the units
    good = pack_requests([(True, [([i % 100], msgs[i], sigs[i].tobytes())]) for i in range(n)])
    v, st = gpu.verify_packed(good)
    assert list(v) == [1] * n and st.merged_check == 1


def test_kat3_mainnet_points_gpu_decode(gpu, golden, oracle, table):
    """KAT-3: the real mainnet G2 points of backfill/blocks.json through the GPU decoder:
    bit-exact uncompressed coordinates and G2 membership (bls_gpu_g2_decompress), then
    through the verify path's own decode + psi subgroup test (k_pre + k_pset, every
    packing): a decodable in-group point that is not this set's signature gives false,
    never an error code."""
    pts = golden["kat3_g2_points"]
    comp = b"".join(bytes.fromhex(p["compressed"]) for p in pts)
    out, codes = gpu.g2_decompress(comp, validate=True)
    assert list(codes) == [0] * len(pts)
    assert [o.tobytes().hex() for o in out] == [p["uncompressed"] for p in pts]
    # aggregator.test.ts:70's bruteforced signature: the oracle's code (parity unpinned)
    unp = golden["kat3_unpinned"]
    _, codes = gpu.g2_decompress(b"".join(bytes.fromhex(u["compressed"]) for u in unp), validate=True)
    assert list(codes) == [u["code"] for u in unp]
    # the oracle-derived negatives through the same entry point
    cases = golden["sig_decode"]
    _, codes = gpu.g2_decompress(b"".join(bytes.fromhex(c["bytes"]) for c in cases), validate=True)
    assert list(codes) == [c["code"] for c in cases]
    # verify path: 1-set requests, and one large batchable call so the packed kernels run
    sks = _keys(oracle, 1)
    m = _h(b"kat3")
    reqs = [(False, [([0], m, bytes.fromhex(p["compressed"]))]) for p in pts]
    v, _ = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == [0] * len(pts)
    sig = gpu.sign(sks[0], m)[0].tobytes()
    big = [(True, [([0], m, sig)])] * 600
    for k, p in enumerate(pts):
        big[37 * k + 5] = (True, [([0], m, bytes.fromhex(p["compressed"]))])
    pb = pack_requests(big)
    want = [0 if (i - 5) % 37 == 0 and (i - 5) // 37 < len(pts) else 1 for i in range(600)]
    for name, (v, _) in _run_all_paths(gpu, pb).items():
        assert list(v) == want, name


def test_verify_many_matches_separate_calls(gpu, oracle, table):
    """bls_gpu_verify_many: several worker messages in one device pass give each message
    the verdicts and chunking of its own bls_gpu_verify call (worker.ts:56 chunks per
    message): messages of 40 / 17 / 33 batchable requests (chunk counts not multiples of
    16 across the joined list), one with a non-batchable request, invalid sets in two,
    a 32-byte signature in one; totals of the stats equal the sums; a message with raw
    pubkeys (deserializeSet per message) runs on its own."""
    sks = _keys(oracle, 16)
    sizes = [40, 17, 33]
    msgs = [[_h(b"many%d-%d" % (k, i)) for i in range(n)] for k, n in enumerate(sizes)]
    flat = [m for ms in msgs for m in ms]
    sigs = gpu.sign(b"".join(sks[j % 16] for j in range(len(flat))), b"".join(flat))
    pbs, j = [], 0
    bad = {(0, 7), (2, 30)}
    for k, n in enumerate(sizes):
        reqs = []
        for i in range(n):
            m = msgs[k][i] if (k, i) not in bad else _h(b"tampered%d-%d" % (k, i))
            s = sigs[j].tobytes() if (k, i) != (1, 3) else bytes(32)
            reqs.append((not (k == 2 and i == 5), [([j % 16], m, s)]))
            j += 1
        pbs.append(pack_requests(reqs))
    sep = [gpu.verify_packed(pb) for pb in pbs]
    many, st = gpu.verify_many(pbs)
    for (v, _), w in zip(sep, many):
        assert list(v) == list(w)
    assert many[0][7] == 0 and many[2][30] == 0 and many[1][3] == -CODE_INVALID_SIZE
    assert st.n_chunks == sum(s.n_chunks for _, s in sep)
    assert st.batch_retries == sum(s.batch_retries for _, s in sep)
    assert st.batch_sigs_success == sum(s.batch_sigs_success for _, s in sep)
    # a raw-pubkey message among them: verified on its own, same verdicts
    raw, _ = gpu.aggregate_pubkeys([[0], [1]])
    rawpb = pack_requests([(True, [(raw[0], msgs[0][0], sigs[0].tobytes())]),
                           (True, [(raw[1], msgs[0][1], sigs[1].tobytes())])])
    many2, _ = gpu.verify_many([pbs[0], rawpb])
    assert list(many2[0]) == list(sep[0][0]) and list(many2[1]) == [1, 1]


def test_verify_many_merged_signature_sum_fails(gpu, oracle, table, verify_path):
    """bls_gpu_verify_many with every request batchable across four messages (the
    bench's pass shape): the merged check (one final exponentiation over the pass, one
    summed signature pairing) runs over the joined messages; one invalid set makes it
    fail (merged_check == 2), each chunk's signature sum is rebuilt and paired, and every
    message still gets the verdicts and stats of its own call (worker.ts:56-88)."""
    sks = _keys(oracle, 16)
    sizes = [64, 48, 80, 33]
    msgs = [[_h(b"mmany%d-%d" % (k, i)) for i in range(n)] for k, n in enumerate(sizes)]
    flat = [m for ms in msgs for m in ms]
    sigs = gpu.sign(b"".join(sks[j % 16] for j in range(len(flat))), b"".join(flat))
    pbs, j = [], 0
    for k, n in enumerate(sizes):
        reqs = []
        for i in range(n):
            m = msgs[k][i] if (k, i) != (2, 41) else _h(b"mtampered")
            reqs.append((True, [([j % 16], m, sigs[j].tobytes())]))
            j += 1
        pbs.append(pack_requests(reqs))
    sep = [gpu.verify_packed(pb) for pb in pbs]
    many, st = gpu.verify_many(pbs)
    for (v, _), w in zip(sep, many):
        assert list(v) == list(w)
    assert many[2][41] == 0 and sum(int((w == 1).sum()) for w in many) == sum(sizes) - 1
    assert st.merged_check == 2
    exp = [_expected_stats(oracle, [0 if (k, i) == (2, 41) else 1 for i in range(n)]) for k, n in enumerate(sizes)]
    assert st.batch_retries == sum(e[0] for e in exp) and st.batch_sigs_success == sum(e[1] for e in exp)
    # all valid: the merged check passes over the joined messages
    good = []
    j = 0
    for k, n in enumerate(sizes):
        good.append(pack_requests([(True, [([(j + i) % 16], msgs[k][i], sigs[j + i].tobytes())]) for i in range(n)]))
        j += n
    many, st = gpu.verify_many(good)
    assert all((w == 1).all() for w in many) and st.merged_check == 1


@pytest.mark.parametrize("n,bad", [(80, 41), (128, 70), (256, 130), (80, 1), (80, 79)])
def test_failed_chunk_requests_verified_alone(gpu, oracle, table, n, bad):
    """One invalid set in a middle chunk: the merged check fails, the chunk fails, and
    its 16 requests are verified alone (worker.ts:81-87) -- every other request of the
    chunk is true.  Regression: the split SIMT Miller loops (kernels/k_mlq.hip k_mlf)
    read the product-domain table past its end for the individual requests' signature
    sums and paired two requests into one f, so at these sizes every request of the
    failed chunk came back false."""
    sks = _keys(oracle, 16)
    msgs = [_h(b"alone%d-%d" % (n, i)) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))
    reqs = [(True, [([i % 16], msgs[i] if i != bad else _h(b"alone-x"), sigs[i].tobytes())]) for i in range(n)]
    expect = [0 if i == bad else 1 for i in range(n)]
    v, st = gpu.verify_packed(pack_requests(reqs))
    assert list(v) == expect
    retries, ok = _expected_stats(oracle, expect)
    assert (st.batch_retries, st.batch_sigs_success, st.merged_check) == (retries, ok, 2)


def test_failed_chunks_group_tested(gpu, oracle, table, verify_path):
    """Failed chunks are group-tested (bls_gpu.hip verify_groups: the test of all the
    chunk's requests beside its bit-index groups, each group's final exponentiation also
    compared with the whole's, so a single invalid request is decoded in one round, else
    every request alone): one
    invalid request at the first / a middle / the last position, two in one chunk (the
    every-request-alone pass), an undecodable signature with every other request valid
    (the group of the rest passes), an undecodable one next to an invalid one, and the
    same with chunks of 5 requests.  Verdicts and worker counters are the reference's."""
    n = 1024
    sks = _keys(oracle, 16)
    msgs = [_h(b"gt-%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))
    bad = {16 + 0, 32 + 7, 48 + 15, 64 + 3, 64 + 12, 96 + 9, 1000}
    undecodable = {80 + 4, 96 + 2}
    for per_req in (1, 3):  # single-set requests (chunks of 16) and 3-set requests (chunks of 5-6)
        reqs, expect = [], []
        for r in range(n // per_req):
            ss, code = [], 1
            for i in range(r * per_req, (r + 1) * per_req):
                sig = sigs[i].tobytes()
                if i in bad:
                    sig = sigs[(i + 1) % n].tobytes()
                    code = min(code, 0) if code >= 0 else code
                if i in undecodable:
                    sig, code = bytes(96), -CODE_BAD_ENCODING
                ss.append(([i % 16], msgs[i], sig))
            reqs.append((True, ss))
            expect.append(code)
        from lodestar_amd._abi import DEBUG_GROUP_TEST

        for flags in (0, DEBUG_GROUP_TEST):
            try:
                gpu.set_debug_flags(flags)
                v, st = gpu.verify_packed(pack_requests(reqs))
            finally:
                gpu.set_debug_flags(0)
            assert list(v) == expect, (per_req, flags)
            if per_req == 1:
                retries, ok = _expected_stats(oracle, expect)
                assert (st.batch_retries, st.batch_sigs_success) == (retries, ok)


def test_msm_signature_sum_matches_chains(gpu, oracle, table, verify_path):
    """The Pippenger merged signature sum (BLS_DEBUG_MSM, kernels/k_msm.hip) gives the
    verdicts and worker stats of the per-set [r] sig chains: 2,048 batchable sets (buckets
    of several segments), all valid (the merged check passes on the MSM sum), then with
    wrong signatures and an undecodable one (the MSM sum fails the merged check, the
    chunks' own sums are rebuilt from k_chain role 2)."""
    from lodestar_amd._abi import DEBUG_MSM

    if verify_path != "sigagg":
        pytest.skip("the MSM replaces the aggregated path's signature sum")
    n = 2048
    sks = _keys(oracle, 16)
    msgs = [_h(b"msm%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))
    for bad in ((), (5, 700, 2047)):
        reqs, expect = [], []
        for i in range(n):
            sig, code = sigs[i].tobytes(), 1
            if i in bad:
                sig, code = sigs[(i + 1) % n].tobytes(), 0
            if bad and i == 100:
                sig, code = bytes(96), -CODE_BAD_ENCODING
            reqs.append((True, [([i % 16], msgs[i], sig)]))
            expect.append(code)
        pb = pack_requests(reqs)
        ref_v, ref_st = gpu.verify_packed(pb)
        try:
            gpu.set_debug_flags(DEBUG_MSM)
            v, st = gpu.verify_packed(pb)
        finally:
            gpu.set_debug_flags(0)
        assert list(v) == expect == list(ref_v)
        assert st.merged_check == ref_st.merged_check == (2 if bad else 1)
        retries, ok = _expected_stats(oracle, expect)
        assert (st.batch_retries, st.batch_sigs_success) == (ref_st.batch_retries, ref_st.batch_sigs_success) == (retries, ok)


@pytest.mark.parametrize("per_lane", [1, 2, 4, 3])
def test_mlf_items_per_lane(gpu, oracle, table, verify_path, per_lane):
    """The f side of the split Miller loops with 1, 2 or 4 items per lane or one item per
    two lanes (3 = MLF_PAIR, k_mlf2) (the library picks by the sets in flight;
    BLS_DEBUG_MLF_PL forces it), with and without the
    Pippenger signature sum: invalid sets at a chunk's first, middle and last position and
    in the last chunk, and an undecodable signature, so lanes whose items do not all share
    a product domain or are not all live run them one by one; the merged check fails,
    each chunk is checked, the failed chunks' requests are verified alone."""
    from lodestar_amd._abi import DEBUG_MLF_PL, DEBUG_MSM

    if verify_path != "sigagg":
        pytest.skip("the split SIMT Miller loops run on the aggregated path")
    n = 1030  # not a multiple of 4: the last lane holds fewer items
    sks = _keys(oracle, 16)
    msgs = [_h(b"mlfpl%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))
    bad = {3, 15, 16, 517, 1029}
    for with_bad in (False, True):
        reqs, expect = [], []
        for i in range(n):
            sig, code = sigs[i].tobytes(), 1
            if with_bad and i in bad:
                sig, code = sigs[(i + 1) % n].tobytes(), 0
            if with_bad and i == 600:
                sig, code = bytes(96), -CODE_BAD_ENCODING
            reqs.append((True, [([i % 16], msgs[i], sig)]))
            expect.append(code)
        pb = pack_requests(reqs)
        retries, ok = _expected_stats(oracle, expect)
        for extra in (0, DEBUG_MSM):
            try:
                gpu.set_debug_flags(DEBUG_MLF_PL(per_lane) | extra)
                v, st = gpu.verify_packed(pb)
            finally:
                gpu.set_debug_flags(0)
            assert list(v) == expect, (per_lane, extra)
            assert st.merged_check == (2 if with_bad else 1)
            assert (st.batch_retries, st.batch_sigs_success) == (retries, ok)
            assert (st.pass_shape >> 8) & 0xFF == per_lane and (st.pass_shape & 1) == (1 if extra else 0)


def test_merged_check_skipped_after_failing_pass(gpu, oracle, table, verify_path):
    """A context whose pass failed its merged check checks its next pass's chunks straight
    away (bls_gpu.hip merged_skip_after_fail: merged_check 3, each chunk's own signature
    sum paired in the pass), until a pass whose chunks all pass; verdicts and the worker
    counters are those of the chunked worker either way (worker.ts:56-88)."""
    from lodestar_amd._abi import DEBUG_SIGAGG_OFF, DEBUG_SIGAGG_ON

    n = 96
    sks = _keys(oracle, 16)
    msgs = [_h(b"skip%d" % i) for i in range(n)]
    sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))

    def call(bad):
        reqs = [(True, [([i % 16], msgs[i] if i not in bad else _h(b"skip-x"), sigs[i].tobytes())]) for i in range(n)]
        expect = [0 if i in bad else 1 for i in range(n)]
        v, st = gpu.verify_packed(pack_requests(reqs))
        assert list(v) == expect
        assert (st.batch_retries, st.batch_sigs_success) == _expected_stats(oracle, expect)
        return st.merged_check

    saved = gpu.base_debug_flags
    gpu.base_debug_flags = DEBUG_SIGAGG_ON if verify_path == "sigagg" else DEBUG_SIGAGG_OFF
    try:
        gpu.set_debug_flags(0)
        call(set())  # whatever the context's history, a passing pass leaves the merged check on
        assert [call({5}), call({40, 41}), call({90}), call(set()), call(set()), call({7})] == [2, 3, 3, 3, 1, 2]
    finally:
        gpu.base_debug_flags = saved
        gpu.set_debug_flags(0)
