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
def progs(coop_programs):
    return coop_programs


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


def test_fin_final_exponentiation(progs, oracle):
    pg, consts = progs
    rng = random.Random(3)
    q = oracle.E2.mul(oracle.G2, rng.randrange(1, 1 << 64))
    pp = oracle.E1.mul(oracle.G1, rng.randrange(1, 1 << 64))
    f0 = oracle.f12_mul(rand12(rng), oracle.miller_loop(pp, q))
    fr = [0] * GC.FRAME
    put12(fr, GC.F, f0)
    simulate(pg["fin_fe1"], fr, consts)
    fr[GC.INV_OUT] = pow(fr[GC.INV_IN], P - 2, P)
    simulate(pg["fin_fe2"], fr, consts)
    assert get12(fr, GC.F) == oracle.final_exponentiation(f0, hard_multiple=3)
