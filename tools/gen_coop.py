#!/usr/bin/env python3
"""Cooperative-kernel programs: the BLS12-381 tower, curve and pairing formulas as
Fp circuits (tools/circuits.py), scheduled for one 64-lane wavefront per task and
emitted as the binary table lodestar_amd/_native/coop_tables.bin that the HIP
interpreter (lodestar_amd/csrc/bls/coop.hpp) executes.

Frame layouts (slot = one Fp; Fp12 / G2 registers in the memory order of the C++
structs in field.hpp / curve.hpp so global <-> LDS copies are straight):

  "fin" frame (chunk / per-request finalisation, k_fin_coop):
    F  0..11   Fp12 accumulator          G  12..23  Fp12 operand (f_i)
    40 INV_IN, 41 INV_OUT (lane-0 inversion)   E 42..49  saved easy-part values
    temporaries 54..FRAME-1

  "pset" frame: see tools/gen_pset.py.

    python tools/gen_coop.py   (run by lodestar_amd/build.py)
"""
from __future__ import annotations

import struct
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from circuits import (  # noqa: E402
    LANES, OP_LIN, OP_MUL, P, ZCHECK, Circuit, ConstBank, Lin, Program, schedule,
)

X_ABS = 0xD201000000010000
FRAME = 256
FRAME2 = 380   # frame of the 2-set programs (kernels/k_pset.hip, CoopLdsN<COOP_FRAME2>; 2 waves/SIMD)
FRAME3 = 640   # frame of the 3-set programs (CoopLdsN<COOP_FRAME3>)
MONT_R = 1 << 384

# "fin" frame registers
F, G, S, R, Q = 0, 12, 24, 30, 36
INV_IN, INV_OUT = 40, 41
E = 42
HR = 50   # H (2 slots) and S2 - S1 (2 slots) of the last G2 addition



# ----------------------------------------------------------------------------
# tower over Lin (same formulas as field.hpp)
# ----------------------------------------------------------------------------
class T:
    def __init__(self, c: Circuit):
        self.c = c

    # Fp2 = (c0, c1)
    def f2(self, slot):
        return (Circuit.inp(slot), Circuit.inp(slot + 1))

    def add2(self, a, b):
        return (a[0] + b[0], a[1] + b[1])

    def sub2(self, a, b):
        return (a[0] - b[0], a[1] - b[1])

    def neg2(self, a):
        return (-a[0], -a[1])

    def sc2(self, a, k):
        return (a[0] * k, a[1] * k)

    def conj2(self, a):
        return (a[0], -a[1])

    def xi2(self, a):  # * (1 + u)
        return (a[0] - a[1], a[0] + a[1])

    def mul2(self, a, b):
        m = self.c.mul
        t0 = m(a[0], b[0])
        t1 = m(a[1], b[1])
        t2 = m(a[0] + a[1], b[0] + b[1])
        return (t0 - t1, t2 - t0 - t1)

    def sqr2(self, a):
        m = self.c.mul
        return (m(a[0] + a[1], a[0] - a[1]), m(a[0], a[1]) * 2)

    def mulfp2(self, a, s: Lin):
        return (self.c.mul(a[0], s), self.c.mul(a[1], s))

    def mulc2(self, a, k):  # times the constant Fp2 k = (k0, k1)
        k0, k1 = k[0] % P, k[1] % P
        c = self.c
        if k1 == 0:
            return (c.mul(a[0], c.const(k0)), c.mul(a[1], c.const(k0)))
        t0 = c.mul(a[0], c.const(k0))
        t1 = c.mul(a[1], c.const(k1))
        t2 = c.mul(a[0] + a[1], c.const(k0 + k1))
        return (t0 - t1, t2 - t0 - t1)

    def mat2(self, a):
        return (self.c.mat(a[0]), self.c.mat(a[1]))

    # Fp6 = (c0, c1, c2) over v^3 = xi
    def f6(self, slot):
        return (self.f2(slot), self.f2(slot + 2), self.f2(slot + 4))

    def add6(self, a, b):
        return tuple(self.add2(x, y) for x, y in zip(a, b))

    def sub6(self, a, b):
        return tuple(self.sub2(x, y) for x, y in zip(a, b))

    def neg6(self, a):
        return tuple(self.neg2(x) for x in a)

    def v6(self, a):  # * v
        return (self.xi2(a[2]), a[0], a[1])

    def mul6(self, a, b):
        t0 = self.mul2(a[0], b[0])
        t1 = self.mul2(a[1], b[1])
        t2 = self.mul2(a[2], b[2])
        c0 = self.sub2(self.sub2(self.mul2(self.add2(a[1], a[2]), self.add2(b[1], b[2])), t1), t2)
        c0 = self.add2(self.xi2(c0), t0)
        c1 = self.sub2(self.sub2(self.mul2(self.add2(a[0], a[1]), self.add2(b[0], b[1])), t0), t1)
        c1 = self.add2(c1, self.xi2(t2))
        c2 = self.sub2(self.sub2(self.mul2(self.add2(a[0], a[2]), self.add2(b[0], b[2])), t0), t2)
        c2 = self.add2(c2, t1)
        return (c0, c1, c2)

    def mat6(self, a):
        return tuple(self.mat2(x) for x in a)

    # Fp12 = (A, B) over w^2 = v
    def f12(self, slot):
        return (self.f6(slot), self.f6(slot + 6))

    def mul12(self, a, b):
        t0 = self.mul6(a[0], b[0])
        t1 = self.mul6(a[1], b[1])
        c1 = self.sub6(self.sub6(self.mul6(self.add6(a[0], a[1]), self.add6(b[0], b[1])), t0), t1)
        c0 = self.add6(t0, self.v6(t1))
        return (c0, c1)

    def sqr12(self, a):
        ab = self.mul6(a[0], a[1])
        s = self.mul6(self.add6(a[0], a[1]), self.add6(a[0], self.v6(a[1])))
        c0 = self.sub6(self.sub6(s, ab), self.v6(ab))
        return (c0, self.add6(ab, ab))

    def conj12(self, a):
        return (a[0], self.neg6(a[1]))

    def mat12(self, a):
        return (self.mat6(a[0]), self.mat6(a[1]))

    def coef(self, f, k):  # coefficient of w^k
        return f[k % 2][k // 2]

    def from_coefs(self, cs):
        return ((cs[0], cs[2], cs[4]), (cs[1], cs[3], cs[5]))

    def frob12(self, a):
        cs = [self.conj2(self.coef(a, 0))]
        for k in range(1, 6):
            cs.append(self.mulc2(self.conj2(self.coef(a, k)), FROB1[k]))
        return self.from_coefs(cs)

    def frob2_12(self, a):
        cs = [self.coef(a, 0)]
        for k in range(1, 6):
            g = FROB2[k]
            x = self.coef(a, k)
            cs.append((self.c.mul(x[0], self.c.const(g)), self.c.mul(x[1], self.c.const(g))))
        return self.from_coefs(cs)

    def csqr12(self, f):
        """Granger-Scott cyclotomic squaring (field.hpp fp12_cyclotomic_sqr)."""
        c = [self.coef(f, k) for k in range(6)]

        def fp4(x, y):
            t0 = self.sqr2(x)
            t1 = self.sqr2(y)
            return self.add2(t0, self.xi2(t1)), self.sub2(self.sub2(self.sqr2(self.add2(x, y)), t0), t1)

        a0, a1 = fp4(c[0], c[3])
        b0, b1 = fp4(c[1], c[4])
        d0, d1 = fp4(c[2], c[5])
        n = [None] * 6
        n[0] = self.add2(self.sc2(self.sub2(a0, c[0]), 2), a0)
        n[3] = self.add2(self.sc2(self.add2(a1, c[3]), 2), a1)
        xd1 = self.xi2(d1)
        n[1] = self.add2(self.sc2(self.add2(xd1, c[1]), 2), xd1)
        n[4] = self.add2(self.sc2(self.sub2(d0, c[4]), 2), d0)
        n[2] = self.add2(self.sc2(self.sub2(b0, c[2]), 2), b0)
        n[5] = self.add2(self.sc2(self.add2(b1, c[5]), 2), b1)
        return self.from_coefs(n)

    def csqr12_pipe(self, f_lin, f_mat):
        """csqr12 for a squaring chain at one product step per squaring: the products take
        their operands from f_lin (the previous squaring's output as an unmaterialised
        combination of its products and the materialised value before it), the output's
        -2 c / +2 c terms reference f_mat (f materialised, computed beside these products),
        so the materialisation of each output runs in the next squaring's product step
        instead of a step of its own."""
        c = [self.coef(f_lin, k) for k in range(6)]
        m = [self.coef(f_mat, k) for k in range(6)]

        def fp4(x, y):
            t0 = self.sqr2(x)
            t1 = self.sqr2(y)
            return self.add2(t0, self.xi2(t1)), self.sub2(self.sub2(self.sqr2(self.add2(x, y)), t0), t1)

        a0, a1 = fp4(c[0], c[3])
        b0, b1 = fp4(c[1], c[4])
        d0, d1 = fp4(c[2], c[5])
        n = [None] * 6
        n[0] = self.sub2(self.sc2(a0, 3), self.sc2(m[0], 2))
        n[3] = self.add2(self.sc2(a1, 3), self.sc2(m[3], 2))
        xd1 = self.xi2(d1)
        n[1] = self.add2(self.sc2(xd1, 3), self.sc2(m[1], 2))
        n[4] = self.sub2(self.sc2(d0, 3), self.sc2(m[4], 2))
        n[2] = self.sub2(self.sc2(b0, 3), self.sc2(m[2], 2))
        n[5] = self.add2(self.sc2(b1, 3), self.sc2(m[5], 2))
        return self.from_coefs(n)

    def mul_line(self, f, l0, l2, l3):
        """f * (l0 + l2 w^2 + l3 w^3) (field.hpp fp12_mul_line)."""
        def mul01(a, d0, d1):
            a0d0 = self.mul2(a[0], d0)
            a1d1 = self.mul2(a[1], d1)
            c0 = self.add2(a0d0, self.xi2(self.mul2(a[2], d1)))
            c1 = self.sub2(self.sub2(self.mul2(self.add2(a[0], a[1]), self.add2(d0, d1)), a0d0), a1d1)
            c2 = self.add2(a1d1, self.mul2(a[2], d0))
            return (c0, c1, c2)

        def mul1(a, d1):
            return (self.xi2(self.mul2(a[2], d1)), self.mul2(a[0], d1), self.mul2(a[1], d1))

        aa = mul01(f[0], l0, l2)
        bb = mul1(f[1], l3)
        c1 = self.sub6(self.sub6(mul01(self.add6(f[0], f[1]), l0, self.add2(l2, l3)), aa), bb)
        c0 = self.add6(aa, self.v6(bb))
        return (c0, c1)


def _f2pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = ((r[0] * a[0] - r[1] * a[1]) % P, (r[0] * a[1] + r[1] * a[0]) % P)
        a = ((a[0] * a[0] - a[1] * a[1]) % P, (2 * a[0] * a[1]) % P)
        e >>= 1
    return r


FROB1 = {k: _f2pow((1, 1), k * (P - 1) // 6) for k in range(1, 6)}
FROB2 = {k: _f2pow((1, 1), k * (P * P - 1) // 6)[0] for k in range(1, 6)}
G1X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
B2X12 = (12, 12)   # 3 b' = 12 (1 + u)


def out12(c: Circuit, base: int, f):
    for k in range(2):
        for j in range(3):
            for i in range(2):
                c.out(base + 6 * k + 2 * j + i, f[k][j][i])


def out2(c: Circuit, base: int, a):
    c.out(base, a[0])
    c.out(base + 1, a[1])


# ----------------------------------------------------------------------------
# curve formulas
# ----------------------------------------------------------------------------
def g2_dbl_jac(t: T, X, Y, Z):
    """dbl-2009-l (curve.hpp jac_dbl)."""
    a = t.sqr2(X)
    b = t.sqr2(Y)
    cc = t.sqr2(b)
    d = t.sc2(t.sub2(t.sub2(t.sqr2(t.add2(X, b)), a), cc), 2)
    e = t.sc2(a, 3)
    f = t.sqr2(e)
    x3 = t.mat2(t.sub2(f, t.sc2(d, 2)))
    y3 = t.sub2(t.mul2(e, t.sub2(d, x3)), t.sc2(cc, 8))
    z3 = t.sc2(t.mul2(Y, Z), 2)
    return x3, y3, z3


def g2_add_jac(t: T, X1, Y1, Z1, X2, Y2, Z2, zcheck=True, hr_out=None):
    """add-2007-bl (curve.hpp jac_add, generic branch); zero-checks H and, when
    hr_out is given, writes H and S2 - S1 there for the exact exceptional-case test."""
    z1z1 = t.sqr2(Z1)
    z2z2 = t.sqr2(Z2)
    u1 = t.mul2(X1, z2z2)
    u2 = t.mul2(X2, z1z1)
    s1 = t.mul2(t.mul2(Y1, Z2), z2z2)
    s2 = t.mul2(t.mul2(Y2, Z1), z1z1)
    h = t.mat2(t.sub2(u2, u1))
    if zcheck:
        t.c.zcheck(h[0])
        t.c.zcheck(h[1])
    if hr_out is not None:
        out2(t.c, hr_out, h)
        out2(t.c, hr_out + 2, t.sub2(s2, s1))
    r = t.sc2(t.sub2(s2, s1), 2)
    i = t.sqr2(t.sc2(h, 2))
    j = t.mul2(h, i)
    v = t.mul2(u1, i)
    x3 = t.sub2(t.sub2(t.sqr2(r), j), t.sc2(v, 2))
    x3 = t.mat2(x3)
    y3 = t.sub2(t.mul2(r, t.sub2(v, x3)), t.sc2(t.mul2(s1, j), 2))
    z3 = t.mul2(t.sub2(t.sub2(t.sqr2(t.add2(Z1, Z2)), z1z1), z2z2), h)
    return x3, y3, z3


def miller_dbl(t: T, Tx, Ty, Tz):
    """Doubling step on the projective twist point (pairing.hpp miller_dbl_step),
    scaled by 4 to avoid halvings: returns the new T and line coefficients (i, 3j, -h)."""
    b = t.sqr2(Ty)
    cc = t.sqr2(Tz)
    xy = t.mul2(Tx, Ty)
    j = t.sqr2(Tx)
    h = t.sub2(t.sub2(t.sqr2(t.add2(Ty, Tz)), b), cc)
    e = t.xi2(t.sc2(cc, 12))           # 3 b' c = 12 (1 + u) c
    f = t.sc2(e, 3)
    e2 = t.sqr2(e)
    nx = t.sc2(t.mul2(xy, t.sub2(b, f)), 2)         # 4 * (xy/2)(b - f)
    ny = t.sub2(t.sqr2(t.add2(b, f)), t.sc2(e2, 12))  # 4 * (g^2 - 3 e^2)
    nz = t.sc2(t.mul2(b, h), 4)                     # 4 * b h
    return (nx, ny, nz), (t.sub2(e, b), t.sc2(j, 3), t.neg2(h))


def miller_add(t: T, Tx, Ty, Tz, qx, qy):
    """Mixed addition step T += Q (pairing.hpp miller_add_step): new T, (j, -theta, lambda)."""
    theta = t.sub2(Ty, t.mul2(qy, Tz))
    lam = t.sub2(Tx, t.mul2(qx, Tz))
    cc = t.sqr2(theta)
    d = t.sqr2(lam)
    e = t.mul2(lam, d)
    ff = t.mul2(Tz, cc)
    g = t.mul2(Tx, d)
    h = t.sub2(t.add2(e, ff), t.sc2(g, 2))
    nx = t.mul2(lam, h)
    ny = t.sub2(t.mul2(theta, t.sub2(g, h)), t.mul2(e, Ty))
    nz = t.mul2(Tz, e)
    j = t.sub2(t.mul2(theta, qx), t.mul2(lam, qy))
    return (nx, ny, nz), (j, t.neg2(theta), lam)


def miller_loop(t: T, qx, qy, pxz: Lin, py: Lin, pz3: Lin | None):
    """f_{|x|,Q}(P), conjugated; P given as (X Z, Y, Z^3) (pz3 None means 1)."""
    c = t.c
    Tp = (qx, qy, (c.one(), Lin()))
    f = None

    def line(coefs):
        l0, l2, l3 = coefs
        if pz3 is not None:
            l0 = t.mulfp2(l0, pz3)
        return l0, t.mulfp2(l2, pxz), t.mulfp2(l3, py)

    def apply(f, coefs):
        l0, l2, l3 = line(coefs)
        l0, l2, l3 = t.mat2(l0), t.mat2(l2), t.mat2(l3)
        if f is None:
            z = (Lin(), Lin())
            return ((l0, l2, z), (z, l3, z))
        return t.mat12(t.mul_line(f, l0, l2, l3))

    for i in range(62, -1, -1):
        if f is not None:
            f = t.mat12(t.sqr12(f))
        Tp, coefs = miller_dbl(t, *Tp)
        Tp = tuple(t.mat2(x) for x in Tp)
        f = apply(f, coefs)
        if (X_ABS >> i) & 1:
            Tp, coefs = miller_add(t, *Tp, qx, qy)
            Tp = tuple(t.mat2(x) for x in Tp)
            f = apply(f, coefs)
    return t.conj12(f)


def cexp_x(t: T, f, pipe: bool = True):
    """f^x = conj(f^|x|) for cyclotomic f.  pipe: the squarings as csqr12_pipe (each
    squaring's products read the previous output unmaterialised; its materialisation
    runs beside the next products), so a run of squarings costs one step each."""
    r = f
    if not pipe:
        for i in range(62, -1, -1):
            r = t.mat12(t.csqr12(r))
            if (X_ABS >> i) & 1:
                r = t.mat12(t.mul12(r, f))
        return t.conj12(r)
    r_lin = r_mat = f
    for i in range(62, -1, -1):
        nl = t.csqr12_pipe(r_lin, r_mat)
        r_lin, r_mat = nl, t.mat12(nl)
        if (X_ABS >> i) & 1:
            r_lin = r_mat = t.mat12(t.mul12(r_mat, f))
    return t.conj12(r_mat)


# ----------------------------------------------------------------------------
# programs
# ----------------------------------------------------------------------------
def build_fin(consts: ConstBank) -> list[Program]:
    progs = []
    fin_regs = set(range(0, 54))

    # F = F * G
    c = Circuit("fin_fmul", consts)
    t = T(c)
    out12(c, F, t.mul12(t.f12(F), t.f12(G)))
    progs.append(schedule(c, FRAME, fin_regs))

    # FE part 1: norms down to Fp (Fp12 -> Fp6 -> Fp2 -> Fp)
    c = Circuit("fin_fe1", consts)
    t = T(c)
    f = t.f12(F)
    A, B = f
    n6 = t.mat6(t.sub6(t.mul6(A, A), t.v6(t.mul6(B, B))))
    n0, n1, n2 = n6
    t0 = t.mat2(t.sub2(t.sqr2(n0), t.xi2(t.mul2(n1, n2))))
    t1 = t.mat2(t.sub2(t.xi2(t.sqr2(n2)), t.mul2(n0, n1)))
    t2 = t.mat2(t.sub2(t.sqr2(n1), t.mul2(n0, n2)))
    nn = t.mat2(t.add2(t.mul2(n0, t0), t.xi2(t.add2(t.mul2(n2, t1), t.mul2(n1, t2)))))
    c.out(INV_IN, c.mul(nn[0], nn[0]) + c.mul(nn[1], nn[1]))
    for k, v in enumerate((t0, t1, t2, nn)):
        out2(c, E + 2 * k, v)
    progs.append(schedule(c, FRAME, fin_regs))

    # FE part 2: inverse, easy part, hard part (HHT, result = e^3); F <- result
    c = Circuit("fin_fe2", consts)
    t = T(c)
    f = t.f12(F)
    A, B = f
    w = Circuit.inp(INV_OUT)
    t0, t1, t2, nn = (t.f2(E + 2 * k) for k in range(4))
    nninv = (c.mul(nn[0], w), -c.mul(nn[1], w))
    n6inv = t.mat6((t.mul2(t0, nninv), t.mul2(t1, nninv), t.mul2(t2, nninv)))
    finv = (t.mul6(A, n6inv), t.neg6(t.mul6(B, n6inv)))
    tt = t.mat12(t.mul12(t.conj12(f), t.mat12(finv)))
    tt = t.mat12(t.mul12(t.mat12(t.frob2_12(tt)), tt))
    a = t.mat12(t.mul12(cexp_x(t, tt), t.conj12(tt)))
    a = t.mat12(t.mul12(cexp_x(t, a), t.conj12(a)))
    b = t.mat12(t.mul12(cexp_x(t, a), t.mat12(t.frob12(a))))
    cc = cexp_x(t, t.mat12(cexp_x(t, b)))
    cc = t.mat12(t.mul12(t.mat12(t.mul12(t.mat12(cc), t.mat12(t.frob2_12(b)))), t.conj12(b)))
    t3 = t.mat12(t.mul12(t.mat12(t.csqr12(tt)), tt))
    out12(c, F, t.mul12(cc, t3))
    progs.append(schedule(c, FRAME, fin_regs))
    return progs


# ----------------------------------------------------------------------------
# emitter
# ----------------------------------------------------------------------------
def _le_limbs(v: int) -> bytes:
    return v.to_bytes(48, "little")


GRP_A, GRP_B = 3, 4  # lanes of a product spread over a group (coop.hpp coop_step)


def _split(terms, k):
    """terms in k consecutive parts (the first ones one longer)"""
    q, r = divmod(len(terms), k)
    out, at = [], 0
    for i in range(k):
        n = q + (1 if i < r else 0)
        out.append(terms[at: at + n])
        at += n
    return out


def lane_entries(step, lanes: int = LANES):
    """A step's lane entries (out, kind, a, b) -- out None: the lane writes nothing -- and
    the step's group sizes (gp, gl) for its products and its combinations.

    The interpreter runs one wavefront per task (two for k_pset's Miller loop), alone on
    its SIMD, so a step's time is one lane's instruction stream, and the operand gathers
    are the larger part of it.  A step with spare lanes therefore spreads its ops over
    aligned lane groups: a product over gp = 2 or 4 lanes (the first half gathers operand
    a -- GRP_A, split over gp / 2 lanes --, the second half operand b -- GRP_B --; each half
    adds its partial sums by DPP, the halves swap the reduced operands and every lane
    multiplies; the group's first lane writes), a combination over gl = 2 or 4 lanes (its
    terms split, the partial sums added by DPP, the first lane writes).  gp is the largest
    of 4, 2, 1 with gp x products + combinations <= lanes, then gl the largest with
    gp x products + gl x combinations <= lanes (one lane per op when neither fits)."""
    muls = [op for op in step if op.kind == OP_MUL]
    lins = [op for op in step if op.kind != OP_MUL]
    gp = next((g for g in (4, 2) if muls and g * len(muls) + len(lins) <= lanes), 1)
    longest = max((len(op.a) for op in lins), default=0)
    def lin_start(g):  # combination groups start aligned to their size
        return -(-gp * len(muls) // g) * g
    gl = next((g for g in (4, 2) if lins and longest > g // 2 and lin_start(g) + g * len(lins) <= lanes), 1)
    out = []
    for op in muls:
        if gp == 1:
            out.append((op.out, OP_MUL, op.a, op.b))
            continue
        h = gp // 2
        for k, part in enumerate(_split(op.a, h)):
            out.append((op.out if k == 0 else None, GRP_A, part, []))
        for part in _split(op.b, h):
            out.append((None, GRP_B, part, []))
    out += [(None, 0, [], [])] * (lin_start(gl) - len(out))
    for op in lins:
        for k, part in enumerate(_split(op.a, gl)):
            out.append((op.out if k == 0 else None, OP_LIN, part, []))
    return out, gp, gl


def emit(progs: list[Program], consts: ConstBank, path: Path) -> None:
    steps_bin = bytearray()
    table = bytearray()
    first = 0
    for pg in progs:
        name = pg.name.encode()[:31].ljust(32, b"\0")
        table += name + struct.pack("<IIII", first, len(pg.steps), pg.n_slots, pg.n_mul_steps)
        L = getattr(pg, "lanes", LANES)  # 64 per wavefront the program runs on
        for step in pg.steps:
            assert len(step) <= L
            entries, gp, gl = lane_entries(step, L)
            # per-step (wave-uniform) fields every lane carries: the largest term count of
            # operand a over the lanes that gather it (every op) and of operand b (the
            # unpaired products), and whether each is a single +1 term on all of them --
            # the interpreter's loop bounds and fast paths without a ballot per step
            act = [e for e in entries if e[1] != 0]
            muls = [e for e in entries if e[1] == OP_MUL]
            ma = max((len(e[2]) for e in act), default=0)
            mb = max((len(e[3]) for e in muls), default=0)
            sa = bool(act) and all(len(e[2]) == 1 and e[2][0][1] == 1 for e in act)
            sb = bool(muls) and all(len(e[3]) == 1 and e[3][0][1] == 1 for e in muls)
            flags = int(sa) | int(sb) << 1 | (gp.bit_length() - 1) << 2 | (gl.bit_length() - 1) << 4
            for lane in range(L):
                if lane < len(entries):
                    out, kind, a, b = entries[lane]
                    # zero-checks: 0xFFFF for set 0, 0xFFF0 + s for packed set s >= 1
                    if out is None:
                        out = 0xFFFE
                    elif out == ZCHECK:
                        out = 0xFFFF
                    elif out < ZCHECK:
                        out = 0xFFF0 + (ZCHECK - out)
                else:
                    out, kind, a, b = 0xFFFE, 0, [], []
                assert len(a) <= 8 and len(b) <= 8
                # +-1 terms first, positive before negative: the interpreter skips the
                # multiply / negate work for term positions no lane of the wave needs
                a = sorted(a, key=lambda t: (abs(t[1]) != 1, t[1] < 0))
                b = sorted(b, key=lambda t: (abs(t[1]) != 1, t[1] < 0))
                def refs(lst):
                    # constants follow the program's frame in LDS (CoopLdsN)
                    r = [((pg.n_slots + x[1]) if isinstance(x, tuple) else x) for x, _ in lst]
                    return r + [0] * (8 - len(r))
                def cfs(lst):
                    r = [cf for _, cf in lst]
                    return r + [0] * (8 - len(r))
                steps_bin += struct.pack("<HBBBBBB8H8H8h8h8x", out, kind, len(a), len(b), ma, mb, flags,
                                         *refs(a), *refs(b), *cfs(a), *cfs(b))
        first += len(pg.steps) * (L // LANES)
    assert len(consts.vals) <= 40, "constant bank exceeds COOP_MAX_CONSTS"
    header = struct.pack("<4sIIII", b"BLSC", 4, len(consts.vals), len(progs), first)
    cbin = b"".join(_le_limbs(v * MONT_R % P) for v in consts.vals)
    path.write_bytes(header + cbin + bytes(table) + bytes(steps_bin))


def _curve_constants():
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        import gen_constants as gc
    return (gc.PSI_X, gc.PSI_Y), (gc.ISO_XNUM, gc.ISO_XDEN, gc.ISO_YNUM, gc.ISO_YDEN)


def build_all():
    import gen_pset
    consts = ConstBank()
    psi, iso = _curve_constants()
    progs = build_fin(consts)
    progs += gen_pset.build_pset(consts, T, miller_dbl, miller_add, X_ABS, FRAME, psi, iso)
    # two / three sets packed per wavefront (k_psetn, large batches)
    progs += gen_pset.build_pset(consts, T, miller_dbl, miller_add, X_ABS, FRAME2, psi, iso,
                                 S=2, prefix="pset2")
    progs += gen_pset.build_pset(consts, T, miller_dbl, miller_add, X_ABS, FRAME3, psi, iso,
                                 S=3, prefix="pset3")
    # single-pair Miller loops of the aggregated-signature path as cooperative programs
    # (k_mln, the packings tests force; the default is the SIMT k_mlq / k_mlf): 1 or 2 sets
    # per wavefront in the 256-slot frame
    progs.append(gen_pset.build_ml1(consts, T, miller_dbl, miller_add, X_ABS, FRAME, S=1))
    progs.append(gen_pset.build_ml1(consts, T, miller_dbl, miller_add, X_ABS, FRAME, S=2))
    # the one-set |x| chains as one straight program (kernels/k_pset.hip): the doubling /
    # addition programs in the order of |x|'s bits, so the interpreter's op fetch stays
    # ahead across the 68 chain steps instead of restarting at every program call
    import copy
    dbl = next(p for p in progs if p.name == "pset_dbl_all")
    addx = next(p for p in progs if p.name == "pset_add_x")
    assert dbl.n_slots == addx.n_slots
    steps = []
    for k in range(62, -1, -1):
        steps += dbl.steps
        if (X_ABS >> k) & 1:
            steps += addx.steps
    progs.append(Program("pset_xchain", steps, dbl.n_slots, [], sum(
        1 for st in steps if any(op.kind == OP_MUL for op in st))))
    # the one-set Miller loop laid out for two wavefronts (kernels/k_pset.hip): the same
    # steps, 128 lanes each, so every product finds a lane pair
    ml2 = next(p for p in progs if p.name == "pset_ml2")
    w2 = copy.copy(ml2)
    w2.name, w2.lanes = "pset_ml2_w2", 2 * LANES
    progs.append(w2)
    # the final exponentiation's hard part likewise (kernels/k_fin.hip k_indiv_coop2: a
    # small call's requests verified alone)
    fe2 = next(p for p in progs if p.name == "fin_fe2")
    f2 = copy.copy(fe2)
    f2.name, f2.lanes = "fin_fe2_w2", 2 * LANES
    progs.append(f2)
    return progs, consts


def main(out: str | None = None) -> None:
    progs, consts = build_all()
    path = Path(out) if out else Path(__file__).resolve().parent.parent / "lodestar_amd" / "_native" / "coop_tables.bin"
    path.parent.mkdir(parents=True, exist_ok=True)
    emit(progs, consts, path)
    import json
    summary = {pg.name: {"steps": len(pg.steps), "mul_steps": pg.n_mul_steps,
                         "mul_ops": sum(1 for st in pg.steps for op in st if op.kind == OP_MUL),
                         "lin_ops": sum(1 for st in pg.steps for op in st if op.kind == OP_LIN)}
               for pg in progs}
    path.with_name("coop_programs.json").write_text(json.dumps(summary, indent=1))
    for pg in progs:
        print(f"{pg.name:18s} steps={len(pg.steps):5d} mul_steps={pg.n_mul_steps:5d} "
              f"ops={sum(len(s) for s in pg.steps):7d}", file=sys.stderr)
    print(f"consts={len(consts.vals)} -> {path} ({path.stat().st_size} bytes)", file=sys.stderr)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
