"""Per-set cooperative programs (tools/gen_pset.py) over the step simulator, against
the oracle: H(m) = hash_to_G2 from the two SSWU points, the G2 subgroup test,
r*g1 / r*pk and f_i = ML(r pk, H) ML(-r g1, sig).  CPU only."""
from __future__ import annotations

import random
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))
import gen_coop as GC  # noqa: E402
import gen_pset as PS  # noqa: E402
from circuits import P, simulate  # noqa: E402


@pytest.fixture(scope="module")
def progs(coop_programs):
    return coop_programs


def _frame_for(oracle, msg, sig_pt, pk_pt, zpk):
    u0, u1 = oracle.hash_to_field_fp2(msg, 2, oracle.DST_POP)
    q0 = oracle.map_to_curve_sswu(u0)
    q1 = oracle.map_to_curve_sswu(u1)
    fr = [0] * GC.FRAME
    fr[PS.Q0:PS.Q0 + 4] = [q0[0][0], q0[0][1], q0[1][0], q0[1][1]]
    fr[PS.Q1:PS.Q1 + 4] = [q1[0][0], q1[0][1], q1[1][0], q1[1][1]]
    fr[PS.SIG:PS.SIG + 4] = [sig_pt[0][0], sig_pt[0][1], sig_pt[1][0], sig_pt[1][1]]
    fr[PS.PK:PS.PK + 3] = [pk_pt[0] * zpk * zpk % P, pk_pt[1] * zpk ** 3 % P, zpk]
    return fr


def _inv(v):
    return pow(v, P - 2, P) if v else 0


def _jac(pt, z):
    """affine G1 point -> Jacobian (X, Y, Z) = (x z^2, y z^3, z)"""
    return (pt[0] * z * z % P, pt[1] * z ** 3 % P, z)


def _r_points(oracle, pk, s, rng):
    """[s] g1 and [s] pk as the second wavefront of k_pset hands them over (Jacobian,
    arbitrary Z)"""
    return (_jac(oracle.E1.mul(oracle.G1, s), rng.randrange(1, P)),
            _jac(oracle.E1.mul(pk, s), rng.randrange(1, P)))


def test_pset_valid_set(progs, oracle):
    pg, consts = progs
    rng = random.Random(11)
    sk = rng.randrange(1, oracle.R)
    msg = bytes(rng.randrange(256) for _ in range(32))
    sig = oracle.E2.mul(oracle.hash_to_g2(msg), sk)
    pk = oracle.E1.mul(oracle.G1, sk)
    r = rng.randrange(1, 1 << 64)
    fr = _frame_for(oracle, msg, sig, pk, rng.randrange(1, P))
    flag, in_group = PS.run_pset(pg, consts, fr, *_r_points(oracle, pk, r, rng), simulate, _inv)
    assert not flag and in_group
    H = oracle.hash_to_g2(msg)
    assert ((fr[PS.HQ], fr[PS.HQ + 1]), (fr[PS.HQ + 2], fr[PS.HQ + 3])) == H
    f = [(fr[PS.F + 6 * (w % 2) + 2 * (w // 2)], fr[PS.F + 6 * (w % 2) + 2 * (w // 2) + 1]) for w in range(6)]
    assert oracle.f12_is_one(oracle.final_exponentiation(f, hard_multiple=3))


def test_pset_wrong_message_and_non_subgroup(progs, oracle):
    pg, consts = progs
    rng = random.Random(12)
    sk = rng.randrange(1, oracle.R)
    msg = bytes(rng.randrange(256) for _ in range(32))
    sig = oracle.E2.mul(oracle.hash_to_g2(b"\x01" * 32), sk)   # signs another message
    pk = oracle.E1.mul(oracle.G1, sk)
    fr = _frame_for(oracle, msg, sig, pk, 1)
    flag, in_group = PS.run_pset(pg, consts, fr, *_r_points(oracle, pk, rng.randrange(1, 1 << 64), rng), simulate,
                                 _inv)
    assert not flag and in_group
    f = [(fr[PS.F + 6 * (w % 2) + 2 * (w // 2)], fr[PS.F + 6 * (w % 2) + 2 * (w // 2) + 1]) for w in range(6)]
    assert not oracle.f12_is_one(oracle.final_exponentiation(f, hard_multiple=3))
    # a point of E2 outside G2 (the SSWU image before cofactor clearing)
    u0, _ = oracle.hash_to_field_fp2(b"x" * 32, 2, oracle.DST_POP)
    off = oracle.iso_map(oracle.map_to_curve_sswu(u0))
    assert not oracle.g2_in_subgroup(off)
    fr = _frame_for(oracle, msg, off, pk, 1)
    flag, in_group = PS.run_pset(pg, consts, fr, *_r_points(oracle, pk, 5, rng), simulate, _inv)
    assert not in_group


@pytest.mark.parametrize("S", [2, 3])
def test_psetn_sets_per_wavefront(progs, oracle, S):
    """The packed programs (k_psetn<S>, S sets per wavefront): valid sets next to a set
    whose signature signs another message; each part of the frame gets its own f_i and
    flags (S = 3 caught an output the scheduler hoisted into a slot the last program
    also uses for temporaries)."""
    pg, consts = progs
    rng = random.Random(13 + S)
    frame = [0] * (GC.FRAME2 if S == 2 else GC.FRAME3)
    rs, expect_one = [], []
    for s in range(S):
        good = s != 1
        sk = rng.randrange(1, oracle.R)
        msg = bytes(rng.randrange(256) for _ in range(32))
        sig = oracle.E2.mul(oracle.hash_to_g2(msg if good else b"\x02" * 32), sk)
        pk = oracle.E1.mul(oracle.G1, sk)
        fr = _frame_for(oracle, msg, sig, pk, rng.randrange(1, P))
        o = PS.SET_SLOTS * s
        frame[o:o + PS.SET_SLOTS] = fr[:PS.SET_SLOTS]
        rs.append(_r_points(oracle, pk, rng.randrange(1, 1 << 64), rng))
        expect_one.append(good)
    flag, in_group = PS.run_psetn(pg, consts, frame, rs, simulate, _inv)
    assert flag == 0 and in_group == [True] * S
    for s in range(S):
        o = PS.SET_SLOTS * s + PS.F
        f = [(frame[o + 6 * (w % 2) + 2 * (w // 2)], frame[o + 6 * (w % 2) + 2 * (w // 2) + 1]) for w in range(6)]
        assert oracle.f12_is_one(oracle.final_exponentiation(f, hard_multiple=3)) == expect_one[s]
