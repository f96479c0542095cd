"""The HIP kernels' math compiled for the CPU (tests/native/hostsim.cpp) against the
oracle and the golden fixtures -- runs without a GPU.  The device build differs only
in fp_mul (the 28-bit-digit product, checked here on raw limbs by
test_fp_mul_d28_lazy, and on the GPU by tests/test_gpu_parity.py)."""
from __future__ import annotations

import ctypes
import hashlib
import random

import numpy as np

from tests._codec import P, b48, bf2, bf12, bg2, f2b, f12b, fp, g1b, g2b


def _buf(n):
    return ctypes.create_string_buffer(n)


def test_fp_ops(hostsim):
    rng = random.Random(1)
    o = _buf(48)
    for _ in range(100):
        a, b = rng.randrange(P), rng.randrange(P)
        hostsim.hs_fp_mul(b48(a), b48(b), o)
        assert fp(o.raw) == a * b % P
        hostsim.hs_fp_sub(b48(a), b48(b), o)
        assert fp(o.raw) == (a - b) % P
    hostsim.hs_fp_inv(b48(12345), o)
    assert fp(o.raw) * 12345 % P == 1


def test_fp_mul_d28_lazy(hostsim):
    """The device Montgomery product (28-bit digits, field.hpp fp_mul_d28_lazy /
    fp_sqr_d28_lazy) on raw limbs: a * b / 2^384 mod p, output < 2p for inputs < 3p,
    including the extremes of the lazy range."""
    rng = random.Random(28)
    o = _buf(48)
    rinv = pow(2, -384, P)
    vals = [0, 1, P - 1, P, 2 * P - 1, 3 * P - 1, 2 ** 382, 3 * P - 2 ** 200]
    vals += [rng.randrange(3 * P) for _ in range(300)]
    for k, a in enumerate(vals):
        b = vals[(7 * k + 3) % len(vals)]
        for sqr in (0, 1):
            hostsim.hs_fp_mul_d28_raw(a.to_bytes(48, "little"), b.to_bytes(48, "little"), o, sqr)
            r = int.from_bytes(o.raw, "little")
            assert r < 2 * P
            assert r % P == (a * (a if sqr else b) * rinv) % P


def test_fp_mul_d28_input_bound(hostsim):
    """The Montgomery product's inputs may reach a b < 2^384 p (output < a b / R + p < 2p):
    fp2_mul_s multiplies a value < 2p by one < 4p (8 p^2)."""
    rng = random.Random(29)
    o = _buf(48)
    rinv = pow(2, -384, P)
    pairs = [(2 * P - 1, 4 * P - 1), (2 * P - 1, 4 * P - 2 ** 100), (P, 4 * P - 1), (0, 4 * P - 1)]
    pairs += [(rng.randrange(2 * P), rng.randrange(4 * P)) for _ in range(300)]
    for a, b in pairs:
        hostsim.hs_fp_mul_d28_raw(a.to_bytes(48, "little"), b.to_bytes(48, "little"), o, 0)
        r = int.from_bytes(o.raw, "little")
        assert r < 2 * P and r % P == (a * b * rinv) % P


def test_fp2_mul_s(hostsim):
    """field.hpp fp2_mul_s: the Fp2 product for operands whose coefficients are unreduced
    sums (< 2p each); canonical output equal to the product of the reduced operands."""
    rng = random.Random(30)
    o = _buf(96)
    rinv = pow(2, -384, P)
    edge = [0, 1, P - 1, P, P + 1, 2 * P - 1, 2 * P - 2, 2 ** 381]
    vals = edge + [rng.randrange(2 * P) for _ in range(200)]
    for k in range(len(vals)):
        a0, a1 = vals[k], vals[(k * 5 + 1) % len(vals)]
        b0, b1 = vals[(k * 11 + 2) % len(vals)], vals[(k * 3 + 4) % len(vals)]
        le = [v.to_bytes(48, "little") for v in (a0, a1, b0, b1)]
        hostsim.hs_fp2_mul_s_raw(le[0] + le[1], le[2] + le[3], o)
        c0, c1 = int.from_bytes(o.raw[:48], "little"), int.from_bytes(o.raw[48:], "little")
        assert c0 < P and c1 < P
        assert c0 == (a0 * b0 - a1 * b1) * rinv % P
        assert c1 == (a0 * b1 + a1 * b0) * rinv % P


def test_fp2_mul_lazy(hostsim):
    """The device Fp2 product with one reduction per coefficient (field.hpp fp2_mul_d28):
    canonical inputs -> canonical (a0 b0 - a1 b1) / R, (a0 b1 + a1 b0) / R, including the
    extremes, and its column offset C2_COL regenerated here: a multiple of p whose every
    column dominates the largest column of a1 b1 for canonical digits."""
    rinv = pow(2, -384, P)
    D = [(1 << 28) - 1] * 13 + [(P - 1) >> 364]
    maxcol = [sum(D[i] * D[k - i] for i in range(14) if 0 <= k - i < 14) for k in range(27)]
    delta = (-sum(c << (28 * k) for k, c in enumerate(maxcol))) % P
    cols = [c + (((delta >> (28 * k)) & ((1 << 28) - 1)) if k < 14 else 0) for k, c in enumerate(maxcol)]
    assert sum(c << (28 * k) for k, c in enumerate(cols)) % P == 0 and max(cols) < 2 ** 61
    src = (__import__("pathlib").Path(__file__).resolve().parent.parent / "lodestar_amd" / "csrc" / "bls" /
           "field.hpp").read_text()
    assert all(("0x%016xull" % c) in src for c in cols)
    rng = random.Random(2)
    o = _buf(96)
    edge = [0, 1, P - 1, P - 2, (P - 1) >> 1, 2 ** 380, P - 2 ** 364]
    vals = edge + [rng.randrange(P) for _ in range(200)]
    for k in range(len(vals)):
        a0, a1 = vals[k], vals[(k * 5 + 1) % len(vals)]
        b0, b1 = vals[(k * 11 + 2) % len(vals)], vals[(k * 3 + 4) % len(vals)]
        le = [v.to_bytes(48, "little") for v in (a0, a1, b0, b1)]
        hostsim.hs_fp2_mul_d28_raw(le[0] + le[1], le[2] + le[3], o)
        c0, c1 = int.from_bytes(o.raw[:48], "little"), int.from_bytes(o.raw[48:], "little")
        assert c0 < P and c1 < P
        assert c0 == (a0 * b0 - a1 * b1) * rinv % P
        assert c1 == (a0 * b1 + a1 * b0) * rinv % P
        hostsim.hs_fp2_sqr_d28_raw(le[0] + le[1], o)
        c0, c1 = int.from_bytes(o.raw[:48], "little"), int.from_bytes(o.raw[48:], "little")
        assert c0 < P and c1 < P
        assert c0 == (a0 * a0 - a1 * a1) * rinv % P
        assert c1 == 2 * a0 * a1 * rinv % P


def test_fp_inv_gcd(hostsim):
    rng = random.Random(7)
    o = _buf(48)
    for a in [1, 2, P - 1, P - 2, 3] + [rng.randrange(1, P) for _ in range(50)]:
        hostsim.hs_fp_inv_gcd(b48(a), o)
        assert fp(o.raw) * a % P == 1
    hostsim.hs_fp_inv_gcd(b48(0), o)
    assert fp(o.raw) == 0


def test_sswu_fast_matches_oracle(hostsim, oracle):
    """map_to_curve_sswu_fast (norm-based branch choice, one Legendre exponentiation)
    equals RFC 9380's map on both branches."""
    rng = random.Random(8)
    o = _buf(192)
    branches = set()
    for k in range(40):
        u = (rng.randrange(P), rng.randrange(P))
        assert hostsim.hs_map_to_curve_sswu_fast(f2b(u), o) == 1
        want = oracle.map_to_curve_sswu(u)
        assert (bf2(o.raw[:96]), bf2(o.raw[96:])) == want
        gx1_square = oracle.f2_is_square(_gx1(oracle, u))
        branches.add(gx1_square)
    assert branches == {True, False}
    # u = 0: den == 0 -> exact-path fallback
    assert hostsim.hs_map_to_curve_sswu_fast(f2b((0, 0)), o) == 0


def test_iso_map_jacobian_matches_oracle(hostsim, oracle):
    """iso_map_jac (k_chain: the 3-isogeny into Jacobian coordinates, no inversion)
    equals RFC 9380's rational map on SSWU outputs, and sends a zero denominator to
    infinity like iso_map_g2."""
    rng = random.Random(11)
    o = _buf(192)
    for _ in range(12):
        u = (rng.randrange(P), rng.randrange(P))
        q = oracle.map_to_curve_sswu(u)
        assert hostsim.hs_iso_map_jac(f2b(q[0]) + f2b(q[1]), o) == 1
        assert (bf2(o.raw[:96]), bf2(o.raw[96:])) == oracle.iso_map(q)
    # a root of the x denominator (x^2 + a1 x + a0 = 0 over Fp2) maps to infinity
    a1, a0 = oracle.ISO_XDEN[1], oracle.ISO_XDEN[0]
    disc = oracle.f2_sub(oracle.f2_mul(a1, a1), oracle.f2_mul((4, 0), a0))
    root = oracle.f2_sqrt(disc)
    if root is not None:
        x = oracle.f2_mul(oracle.f2_sub(root, a1), oracle.f2_inv((2, 0)))
        assert hostsim.hs_iso_map_jac(f2b(x) + f2b((1, 0)), o) == 0


def _gx1(oracle, u):
    Z = oracle.Z_SSWU
    zu2 = oracle.f2_mul(Z, oracle.f2_mul(u, u))
    den = oracle.f2_add(oracle.f2_mul(zu2, zu2), zu2)
    mba = oracle.f2_mul(oracle.f2_neg(oracle.B_ISO), oracle.f2_inv(oracle.A_ISO))
    x1 = oracle.f2_mul(mba, oracle.f2_add(oracle.F2_ONE, oracle.f2_inv(den)))
    return oracle.f2_add(oracle.f2_mul(oracle.f2_add(oracle.f2_mul(x1, x1), oracle.A_ISO), x1), oracle.B_ISO)


def test_fp2_sqrt(hostsim, oracle):
    rng = random.Random(2)
    o = _buf(96)
    for _ in range(20):
        x = (rng.randrange(P), rng.randrange(P))
        ok = hostsim.hs_fp2_sqrt(f2b(x), o)
        assert bool(ok) == (oracle.f2_sqrt(x) is not None)
        if ok:
            assert oracle.f2_mul(bf2(o.raw), bf2(o.raw)) == x
    for x in ((5, 0), (P - 5, 0), (0, 7)):  # the a1 == 0 branch and a0 == 0
        s = oracle.f2_mul(x, x)
        assert hostsim.hs_fp2_sqrt(f2b(s), o) == 1
        assert oracle.f2_mul(bf2(o.raw), bf2(o.raw)) == s


def test_fp12_tower(hostsim, oracle):
    rng = random.Random(3)
    a = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
    b = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
    o = _buf(576)
    hostsim.hs_fp12_mul(f12b(a), f12b(b), o)
    assert bf12(o.raw) == oracle.f12_mul(a, b)
    hostsim.hs_fp12_sqr(f12b(a), o)
    assert bf12(o.raw) == oracle.f12_mul(a, a)
    hostsim.hs_fp12_frob(f12b(a), o)
    assert bf12(o.raw) == oracle.f12_frob(a)
    t = oracle.f12_mul(oracle.f12_conj(a), oracle.f12_inv(a))
    t = oracle.f12_mul(oracle.f12_frob(oracle.f12_frob(t)), t)
    hostsim.hs_fp12_cyclotomic_sqr(f12b(t), o)
    assert bf12(o.raw) == oracle.f12_mul(t, t)


def test_fp12_mul_line2(hostsim):
    """Two sparse line products at once (field.hpp fp12_mul_line2: the lines' product
    first, 23 Fp2 products instead of 26) equal the two products one after the other."""
    rng = random.Random(12)
    o1, o2 = _buf(576), _buf(576)
    for _ in range(20):
        f = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
        ls = [[(rng.randrange(P), rng.randrange(P)) for _ in range(3)] for _ in range(2)]
        hostsim.hs_fp12_mul_line(f12b(f), f2b(ls[0][0]), f2b(ls[0][1]), f2b(ls[0][2]), o1)
        hostsim.hs_fp12_mul_line(o1.raw, f2b(ls[1][0]), f2b(ls[1][1]), f2b(ls[1][2]), o1)
        hostsim.hs_fp12_mul_line2(f12b(f), b"".join(f2b(x) for x in ls[0]), b"".join(f2b(x) for x in ls[1]), o2)
        assert o1.raw == o2.raw


def test_fp12_pair_halves(hostsim):
    """One f over two lanes (k_mlf2, field.hpp fp12_sqr_half_* / fp12_line_half_*): each
    half's products, swapped with the other's, give both halves the full square and the
    full sparse line product."""
    rng = random.Random(14)
    o1, o2 = _buf(576), _buf(2 * 576)
    for _ in range(20):
        f = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
        hostsim.hs_fp12_sqr(f12b(f), o1)
        hostsim.hs_fp12_sqr_pair(f12b(f), o2)
        assert o2.raw[:576] == o2.raw[576:] == o1.raw
        ls = [(rng.randrange(P), rng.randrange(P)) for _ in range(3)]
        hostsim.hs_fp12_mul_line(f12b(f), f2b(ls[0]), f2b(ls[1]), f2b(ls[2]), o1)
        hostsim.hs_fp12_mul_line_pair(f12b(f), f2b(ls[0]), f2b(ls[1]), f2b(ls[2]), o2)
        assert o2.raw[:576] == o2.raw[576:] == o1.raw


def test_group_decode_complement_inference(hostsim):
    """bls_gpu.hip verify_groups' decode of a failed chunk (bls/group_decode.hpp) against a
    model of the tests: each request's final exponentiation is a group element (1 for a
    valid request; a random non-identity one for an invalid), a test's value the product
    over its requests.  With one invalid request the decode names it (the others valid);
    with none it says all valid; with two or more it never names one -- it sends the
    chunk to one test per request -- for every chunk size 1..16 and every position."""
    import itertools

    q = (1 << 61) - 1  # additive model of the target group: value 0 = identity
    rng = random.Random(41)
    vbuf = (ctypes.c_int32 * 8)()
    hostsim.hs_group_decode.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]

    def decode(m, bad):
        val = {b: rng.randrange(1, q) for b in bad}
        whole = sum(val.values()) % q
        nbits = 0
        while m > 1 and (1 << nbits) < m:
            nbits += 1
        for j in range(nbits):
            g = sum(val.get(k, 0) for k in range(m) if (k >> j) & 1) % q
            vbuf[j] = (1 if g == 0 else 0) | (2 if g == whole else 0)
        return hostsim.hs_group_decode(m, nbits, int(whole == 0), ctypes.addressof(vbuf))

    for m in range(1, 17):
        assert decode(m, set()) == m
        for b in range(m):
            assert decode(m, {b}) == b, (m, b)
        for pair in itertools.combinations(range(m), 2):
            assert decode(m, set(pair)) == -1, (m, pair)
        for _ in range(20):
            if m >= 3:
                assert decode(m, set(rng.sample(range(m), rng.randrange(3, m + 1)))) == -1


def test_hash_to_g2_golden(hostsim, golden):
    o = _buf(192)
    for v in golden["hash_to_g2"]:
        hostsim.hs_hash_to_g2(bytes.fromhex(v["msg"]), o)
        assert o.raw.hex() == v["point"]


def test_pairing_matches_oracle_cubed(hostsim, oracle):
    Pp = oracle.E1.mul(oracle.G1, 99)
    Qq = oracle.E2.mul(oracle.G2, 7)
    o = _buf(576)
    hostsim.hs_pairing(g1b(Pp), g2b(Qq), o)
    assert bf12(o.raw) == oracle.final_exponentiation(oracle.miller_loop(Pp, Qq), hard_multiple=3)


def test_sig_decode_cases(hostsim, golden):
    o = _buf(192)
    for case in golden["sig_decode"]:
        raw = bytes.fromhex(case["bytes"])
        code = hostsim.hs_g2_decompress(raw, o)
        if code == 0 and not (raw[0] & 0x40):
            code = 0 if hostsim.hs_g2_in_subgroup(o.raw) else 3
        assert code == case["code"], case["name"]


def test_kat_points(hostsim, golden):
    o = _buf(192)
    for p in golden["kat3_g2_points"]:
        assert hostsim.hs_g2_decompress(bytes.fromhex(p["compressed"]), o) == 0
        assert o.raw.hex() == p["uncompressed"]
        assert hostsim.hs_g2_in_subgroup(o.raw) == 1
    o48 = _buf(48)
    hostsim.hs_sk_to_pk(bytes.fromhex(golden["kat1"]["sk"]), o48)
    assert o48.raw.hex() == golden["kat1"]["pubkey"]
    o96 = _buf(96)
    hostsim.hs_sign(bytes.fromhex(golden["kat1"]["sk"]), bytes.fromhex(golden["kat1"]["signing_root"]), o96)
    assert o96.raw.hex() == golden["kat1"]["signature"]


def _hs_verify(hostsim, reqs, seed=b"\x07" * 32):
    from lodestar_amd._abi import BlsBatch, BlsStats
    from lodestar_amd.native import _ptr, pack_requests

    pb = pack_requests(reqs, seed=seed)
    b = BlsBatch()
    b.n_sets, b.n_reqs = pb.n_sets, pb.n_reqs
    keep = []
    for f in ("req_set_offsets", "req_batchable", "messages", "signatures", "pubkeys", "set_pk_offsets",
              "pk_indices", "signature_lens"):
        a = getattr(pb, f)
        keep.append(a)
        setattr(b, f, _ptr(a))
    s = ctypes.create_string_buffer(seed, 32)
    b.seed = ctypes.cast(s, ctypes.c_void_p)
    v = np.zeros(max(pb.n_reqs, 1), dtype=np.int32)
    st = BlsStats()
    hostsim.hs_verify_batch(ctypes.byref(b), _ptr(v), ctypes.byref(st))
    return list(v[: pb.n_reqs]), st


def test_pipeline_semantics(hostsim, oracle):
    """The kernels' stage bodies, planned and assembled by the same host code as
    bls_gpu_verify, against the reference worker semantics (worker.ts:32-108)."""
    n = 20
    sks = [oracle.interop_secret_key(i) for i in range(n)]
    pks = b""
    for sk in sks:
        o = _buf(48)
        hostsim.hs_sk_to_pk(sk.to_bytes(32, "big"), o)
        pks += o.raw
    hostsim.hs_clear_pubkeys()
    assert hostsim.hs_load_pubkeys(pks, n, 48, None) == n
    msgs = [hashlib.sha256(b"hs%d" % i).digest() for i in range(n)]
    sigs = []
    for sk, m in zip(sks, msgs):
        o = _buf(96)
        hostsim.hs_sign(sk.to_bytes(32, "big"), m, o)
        sigs.append(o.raw)
    sets = [([i], msgs[i], sigs[i]) for i in range(n)]
    reqs = [(True, [s]) for s in sets]
    v, st = _hs_verify(hostsim, reqs)
    assert v == [1] * n and st.n_chunks == 1 and st.batch_retries == 0
    bad = list(reqs)
    bad[3] = (True, [([3], msgs[4], sigs[3])])
    bad[7] = (True, [([7], msgs[7], bytes(32))])
    v, st = _hs_verify(hostsim, bad + [(False, sets[:4]), (False, [])])
    assert v == [1, 1, 1, 0, 1, 1, 1, -8] + [1] * 12 + [1, -10]
    assert st.batch_retries == 1 and st.n_individual == n + 2


def test_deserialize_set_rejects_whole_call(hostsim, oracle):
    """worker.ts:43-46: deserializeSet maps every request of a worker message before any
    verification, outside the try; one raw key that does not decode throws, and the pool
    rejects every job of the message (index.ts:367-374).  The kernels' stage bodies and
    the oracle agree on that (the first bad key in request order names the error)."""
    sk = oracle.interop_secret_key(0)
    pk = oracle.g1_serialize(oracle.sk_to_pk(sk))
    msg = hashlib.sha256(b"deser").digest()
    sig = oracle.g2_compress(oracle.sign(sk, msg))
    good = (pk, msg, sig)
    flag_bit = bytes([0x80]) + pk[1:]                         # compressed flag on a 96-byte key
    off_curve = pk[:48] + (int.from_bytes(pk[48:], "big") ^ 1).to_bytes(48, "big")
    for reqs, code in (
        ([(True, [good]), (False, [good, (flag_bit, msg, sig)]), (False, [])], oracle.E_BAD_ENCODING),
        ([(True, [(off_curve, msg, sig)]), (True, [(flag_bit, msg, sig)])], oracle.E_POINT_NOT_ON_CURVE),
    ):
        v, _ = _hs_verify(hostsim, reqs)
        assert v == [-code] * len(reqs)
        want, retries, ok = oracle.verify_many_signature_sets(reqs)
        assert [-r[1].code for r in want] == v and (retries, ok) == (0, 0)


def test_signing_root_dedup_pre_stage(hostsim):
    """plan_msg_dedup + stage_pre over distinct roots + stage_qdup give every set the
    SSWU points of the per-set pre-stage (committee-shared roots)."""
    import ctypes
    import hashlib

    import numpy as np

    roots = [hashlib.sha256(b"root%d" % k).digest() for k in range(5)]
    order = [3, 0, 3, 1, 4, 0, 0, 2, 3, 4, 1, 3]  # ragged multiplicities, first use out of order
    msgs = b"".join(roots[k] for k in order)
    n = len(order)
    uniq = np.zeros(n, np.uint32)
    rep = np.zeros(n, np.uint32)
    q = np.zeros(n * 8 * 48, np.uint8)
    f = hostsim.hs_pre_dedup_check
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    u = f(msgs, n, uniq.ctypes.data, rep.ctypes.data, q.ctypes.data)
    assert u == 5
    first = {}
    for i, k in enumerate(order):
        first.setdefault(k, i)
    assert list(uniq[:u]) == sorted(first.values())
    assert list(rep) == [first[k] for k in order]
    # all-distinct and all-equal extremes
    assert f(b"".join(roots), 5, uniq.ctypes.data, rep.ctypes.data, q.ctypes.data) == 5
    assert f(roots[2] * 7, 7, uniq.ctypes.data, rep.ctypes.data, q.ctypes.data) == 1
    assert list(rep[:7]) == [0] * 7


def test_windowed_scalar_mul_matches_double_and_add(hostsim):
    """k_chain's [r] sig / [r] pk (curve.hpp jac_mul_u64_w4: a 4-bit window over a
    table of [1..15]P) give the same G1 / G2 elements as double-and-add, for random
    64-bit scalars and the edge ones (0, 1, 15, 16, top nibble 0, 2^60, 2^64 - 1)."""
    hostsim.hs_mul_window_check.restype = ctypes.c_int
    hostsim.hs_mul_window_check.argtypes = [ctypes.c_ulonglong, ctypes.c_int]
    assert hostsim.hs_mul_window_check(20261017, 24) == 0


def test_glv_scalar_mul_matches_full_scalar(hostsim):
    """k_chain's [r] pk / [r] sig as [a]P + [b]endo(P) (curve.hpp jac_mul_glv) equals [k]P
    by double-and-add for k = (a + b mu) mod r, mu = -x^2: the G1 endomorphism sigma and
    -psi^2 on G2 both act as [mu] (the eigenvalue the scalar split relies on)."""
    import random

    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    X = -0xD201000000010000
    mu = (-X * X) % R
    hostsim.hs_glv_check.restype = ctypes.c_int
    hostsim.hs_glv_check.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int]
    rng = random.Random(7)
    cases = [(0, 1), (1, 0), (0xFFFFFFFF, 0xFFFFFFFF), (1, 1), (3, 0), (0, 3)] + \
            [(rng.getrandbits(32), rng.getrandbits(32)) for _ in range(10)]
    for k, (a, b) in enumerate(cases):
        kk = ((a + b * mu) % R).to_bytes(32, "little")
        for g2 in (0, 1):
            assert hostsim.hs_glv_check(a, b, kk, 1000003 + k, g2) == 1, (a, b, g2)
