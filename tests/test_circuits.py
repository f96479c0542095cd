"""The cooperative-kernel programs (tools/gen_coop.py), simulated with the device's
step semantics (tools/circuits.py:simulate), against the oracle's math.  CPU only."""
from __future__ import annotations

import random
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))
import gen_coop as GC  # noqa: E402
from circuits import P, simulate  # noqa: E402


@pytest.fixture(scope="module")
def progs():
    progs, consts = GC.build_all()
    return {p.name: p for p in progs}, consts


def put12(frame, base, f):
    # oracle w-basis coefficients [c0..c5] -> struct order A(c0,c2,c4), B(c1,c3,c5)
    for k in range(2):
        for j in range(3):
            c = f[2 * j + k]
            frame[base + 6 * k + 2 * j] = c[0]
            frame[base + 6 * k + 2 * j + 1] = c[1]


def get12(frame, base):
    return [(frame[base + 6 * (w % 2) + 2 * (w // 2)], frame[base + 6 * (w % 2) + 2 * (w // 2) + 1])
            for w in range(6)]


def rand12(rng):
    return [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]


def to_jac(pt, z):
    (x, y) = pt
    z2 = z
    zz = [(z2[0] * z2[0] - z2[1] * z2[1]) % P, 2 * z2[0] * z2[1] % P]
    from oracle.bls_oracle import f2_mul
    zz = f2_mul(z, z)
    zzz = f2_mul(zz, z)
    return f2_mul(x, zz), f2_mul(y, zzz), z


def test_fin_fmul(progs, oracle):
    pg, consts = progs
    rng = random.Random(1)
    fr = [0] * GC.FRAME
    a, b = rand12(rng), rand12(rng)
    put12(fr, GC.F, a)
    put12(fr, GC.G, b)
    simulate(pg["fin_fmul"], fr, consts)
    assert get12(fr, GC.F) == oracle.f12_mul(a, b)


def test_fin_g2add_and_affine(progs, oracle):
    pg, consts = progs
    rng = random.Random(2)
    p1 = oracle.E2.mul(oracle.G2, rng.randrange(1, 1 << 64))
    p2 = oracle.E2.mul(oracle.G2, rng.randrange(1, 1 << 64))
    fr = [0] * GC.FRAME
    z1 = (rng.randrange(P), rng.randrange(P))
    z2 = (rng.randrange(P), rng.randrange(P))
    for base, pt, z in ((GC.S, p1, z1), (GC.R, p2, z2)):
        X, Y, Z = to_jac(pt, z)
        fr[base:base + 6] = [X[0], X[1], Y[0], Y[1], Z[0], Z[1]]
    flag = simulate(pg["fin_g2add"], fr, consts)
    assert not flag
    simulate(pg["fin_normz"], fr, consts)
    fr[GC.INV_OUT] = pow(fr[GC.INV_IN], P - 2, P)
    simulate(pg["fin_affine"], fr, consts)
    assert ((fr[GC.Q], fr[GC.Q + 1]), (fr[GC.Q + 2], fr[GC.Q + 3])) == oracle.E2.add(p1, p2)
    # H == 0 (P + P) raises the zero-check flag
    X, Y, Z = to_jac(p1, z1)
    fr[GC.S:GC.S + 6] = [X[0], X[1], Y[0], Y[1], Z[0], Z[1]]
    X, Y, Z = to_jac(p1, z2)
    fr[GC.R:GC.R + 6] = [X[0], X[1], Y[0], Y[1], Z[0], Z[1]]
    assert simulate(pg["fin_g2add"], fr, consts)


def test_fin_ml_and_final_exponentiation(progs, oracle):
    pg, consts = progs
    rng = random.Random(3)
    q = oracle.E2.mul(oracle.G2, rng.randrange(1, 1 << 64))
    f0 = rand12(rng)
    fr = [0] * GC.FRAME
    put12(fr, GC.F, f0)
    fr[GC.Q:GC.Q + 4] = [q[0][0], q[0][1], q[1][0], q[1][1]]
    simulate(pg["fin_ml_neg_g1"], fr, consts)
    got_ml = get12(fr, GC.F)
    simulate(pg["fin_fe1"], fr, consts)
    fr[GC.INV_OUT] = pow(fr[GC.INV_IN], P - 2, P)
    simulate(pg["fin_fe2"], fr, consts)
    got = get12(fr, GC.F)
    want = oracle.final_exponentiation(oracle.f12_mul(f0, oracle.miller_loop(oracle.E1.neg(oracle.G1), q)),
                                       hard_multiple=3)
    assert got == want
    # the program's FE alone equals the oracle's FE (x3) on the Miller output
    assert oracle.final_exponentiation(got_ml, hard_multiple=3) == want


def test_fin_g2dbl(progs, oracle):
    pg, consts = progs
    rng = random.Random(4)
    p1 = oracle.E2.mul(oracle.G2, rng.randrange(1, 1 << 64))
    fr = [0] * GC.FRAME
    X, Y, Z = to_jac(p1, (rng.randrange(P), rng.randrange(P)))
    fr[GC.R:GC.R + 6] = [X[0], X[1], Y[0], Y[1], Z[0], Z[1]]
    simulate(pg["fin_g2dbl"], fr, consts)
    simulate(pg["fin_normz"], fr, consts)
    fr[GC.INV_OUT] = pow(fr[GC.INV_IN], P - 2, P)
    simulate(pg["fin_affine"], fr, consts)
    assert ((fr[GC.Q], fr[GC.Q + 1]), (fr[GC.Q + 2], fr[GC.Q + 3])) == oracle.E2.dbl(p1)


def test_set_ml_jacobian_p(progs, oracle):
    """Per-set Miller loop with the G1 point in Jacobian form (line scaled by Z^3)."""
    pg, consts = progs
    rng = random.Random(5)
    q = oracle.E2.mul(oracle.G2, rng.randrange(1, 1 << 64))
    pp = oracle.E1.mul(oracle.G1, rng.randrange(1, 1 << 64))
    z = rng.randrange(1, P)
    fr = [0] * GC.FRAME
    fr[GC.SQ:GC.SQ + 4] = [q[0][0], q[0][1], q[1][0], q[1][1]]
    fr[GC.SP:GC.SP + 3] = [pp[0] * z * z % P, pp[1] * z * z * z % P, z]
    simulate(pg["set_ml"], fr, consts)
    got = get12(fr, GC.SF)
    want = oracle.miller_loop(pp, q)
    assert oracle.final_exponentiation(got, 3) == oracle.final_exponentiation(want, 3)
