"""Per-set cooperative programs ("pset" frame) for the one-wavefront-per-set kernel
(lodestar_amd/csrc/kernels/k_pset.hip).  Imported by tools/gen_coop.py.

The set's work, after the single-lane kernel has produced the two SSWU points
q0, q1 on E2', the decompressed signature and the public key:

  H     = clear_cofactor(iso(q0) + iso(q1))                  (RFC 9380, Budroni-Pintore)
  check = psi(sig) == [x] sig                                 (G2 membership, Scott)
  RG    = [r] g1,   RP = [r] pk                               (64-bit batch scalar)
  f_i   = ML(RP, H) * ML(-RG, sig)                            (two-pair Miller loop)

The random scalar sits on G1 on both sides: e(-g1, r sig) = e(-[r] g1, sig) for sig
in G2 (checked here), so the batch product is the reference's element of GT while
both scalar chains run on G1 (3x cheaper than G2) and sig stays affine for the
Miller loop (one inversion per set, for H only).

The |x| multiplications run left to right, one doubling program per bit for both
chains at once (lanes in parallel) and an addition program at the set bits of |x|.
RG = [s] g1 and RP = [s] pk for the set's batch scalar s come from k_pre's GLV lanes
(kernels/k_pre.hip pre_rpts) and are loaded into the frame with the set's inputs: as
interpreter programs (a 64-bit double-and-add beside the |x| chains) they added ~290
steps to every set's critical path.  Additions zero-check H: an exceptional case
(possible only for adversarial signatures off the subgroup, or with negligible
probability) flags the set for the exact single-lane path.

Frame (slots):
  Q0 0..3  Q1 4..7  SIG 8..11 (affine)  PK 12..14 (G1 Jacobian)
  A 15..20 (cofactor chain [|x|]P)  C 21..26 (subgroup chain [|x|]sig)
  PP 45..50 (P = iso(q0) + iso(q1))  H 51..56  RG 57..59  RP 63..65
  HQ 66..69 (affine)  INV_IN 74  INV_OUT 75  DIFF 76..79 (subgroup test)
  F 80..91 (f_i)  temporaries 92..FRAME-1
"""
from __future__ import annotations

from circuits import Circuit, Lin, schedule

Q0, Q1, SIG, PK = 0, 4, 8, 12
A, C = 15, 21
PP, H, RG, RP = 45, 51, 57, 63
HQ, INV_IN, INV_OUT, DIFF, F = 66, 74, 75, 76, 80
REGS = set(range(0, 92))


class F1:
    """Fp as a one-element field for the generic point formulas."""

    def __init__(self, c: Circuit):
        self.c = c

    def add(self, a, b):
        return a + b

    def sub(self, a, b):
        return a - b

    def neg(self, a):
        return -a

    def sc(self, a, k):
        return a * k

    def mul(self, a, b):
        return self.c.mul(a, b)

    def sqr(self, a):
        return self.c.mul(a, a)

    def mat(self, a):
        return self.c.mat(a)

    def zero(self, a):
        self.c.zcheck(a)

    def reg(self, base):
        return Circuit.inp(base)

    def one(self):
        return self.c.one()

    def out(self, slot, v):
        self.c.out(slot, v)

    width = 1


class F2:
    def __init__(self, t):
        self.t = t
        self.c = t.c

    def add(self, a, b):
        return self.t.add2(a, b)

    def sub(self, a, b):
        return self.t.sub2(a, b)

    def neg(self, a):
        return self.t.neg2(a)

    def sc(self, a, k):
        return self.t.sc2(a, k)

    def mul(self, a, b):
        return self.t.mul2(a, b)

    def sqr(self, a):
        return self.t.sqr2(a)

    def mat(self, a):
        return self.t.mat2(a)

    def zero(self, a):
        self.c.zcheck(a[0])
        self.c.zcheck(a[1])

    def reg(self, base):
        return self.t.f2(base)

    def one(self):
        return (self.c.one(), Lin())

    def out(self, slot, v):
        self.c.out(slot, v[0])
        self.c.out(slot + 1, v[1])

    width = 2


def jac(fo, base):
    w = fo.width
    return (fo.reg(base), fo.reg(base + w), fo.reg(base + 2 * w))


def aff(fo, base):
    w = fo.width
    return (fo.reg(base), fo.reg(base + w))


def out_jac(fo, base, pt):
    w = fo.width
    for k in range(3):
        fo.out(base + k * w, pt[k])


def dbl(fo, p):
    X, Y, Z = p
    a = fo.sqr(X)
    b = fo.sqr(Y)
    cc = fo.sqr(b)
    d = fo.sc(fo.sub(fo.sub(fo.sqr(fo.add(X, b)), a), cc), 2)
    e = fo.sc(a, 3)
    f = fo.sqr(e)
    # no materialisation: the outputs (or the next doubling's operands, inside one
    # program) take the linear combinations directly -- 4 steps instead of 6
    x3 = fo.sub(f, fo.sc(d, 2))
    y3 = fo.sub(fo.mul(e, fo.sub(d, x3)), fo.sc(cc, 8))
    z3 = fo.mul(fo.sc(Y, 2), Z)
    return x3, y3, z3


def add_gen(fo, p, q, check=True):
    """add-2007-bl; zero-checks H (exceptional: P == +-Q or an input at infinity)."""
    X1, Y1, Z1 = p
    X2, Y2, Z2 = q
    z1z1 = fo.sqr(Z1)
    z2z2 = fo.sqr(Z2)
    u1 = fo.mul(X1, z2z2)
    u2 = fo.mul(X2, z1z1)
    s1 = fo.mul(fo.mul(Y1, Z2), z2z2)
    s2 = fo.mul(fo.mul(Y2, Z1), z1z1)
    h = fo.mat(fo.sub(u2, u1))
    if check:
        fo.zero(h)
    r = fo.sc(fo.sub(s2, s1), 2)
    i = fo.sqr(fo.sc(h, 2))
    j = fo.mul(h, i)
    v = fo.mul(u1, i)
    x3 = fo.sub(fo.sub(fo.sqr(r), j), fo.sc(v, 2))
    y3 = fo.sub(fo.mul(r, fo.sub(v, x3)), fo.sc(fo.mul(s1, j), 2))
    z3 = fo.mul(fo.sub(fo.sub(fo.sqr(fo.add(Z1, Z2)), z1z1), z2z2), h)
    return x3, y3, z3  # linear combinations, as dbl's


def add_mixed(fo, p, q, check=True):
    """madd-2007-bl: p Jacobian + q affine; zero-checks H."""
    X1, Y1, Z1 = p
    X2, Y2 = q
    z1z1 = fo.sqr(Z1)
    u2 = fo.mul(X2, z1z1)
    s2 = fo.mul(fo.mul(Y2, Z1), z1z1)
    h = fo.mat(fo.sub(u2, X1))
    if check:
        fo.zero(h)
    hh = fo.sqr(h)
    i = fo.sc(hh, 4)
    j = fo.mul(h, i)
    r = fo.sc(fo.sub(s2, Y1), 2)
    v = fo.mul(X1, i)
    x3 = fo.sub(fo.sub(fo.sqr(r), j), fo.sc(v, 2))
    y3 = fo.sub(fo.mul(r, fo.sub(v, x3)), fo.sc(fo.mul(Y1, j), 2))
    z3 = fo.sub(fo.sub(fo.sqr(fo.add(Z1, h)), z1z1), hh)
    return x3, y3, z3


def neg_pt(fo, p):
    return (p[0], fo.neg(p[1]), p[2])


def psi_jac(t, p, consts_psi):
    cx, cy = consts_psi
    X, Y, Z = p
    return (t.mat2(t.mulc2(t.conj2(X), cx)), t.mat2(t.mulc2(t.conj2(Y), cy)), t.conj2(Z))


def iso_jac(t, x, y, iso):
    """3-isogeny E2' -> E2 in Jacobian form (no inversion):
       Z = xd yd, X = xn xd yd^2, Y = y yn xd^3 yd^2; zero-checks xd and yd (infinity)."""
    xnum, xden, ynum, yden = iso

    def horner(coefs, monic):
        # coefficients low -> high; a monic polynomial lists its leading 1 last
        cs = list(coefs)
        if monic:
            acc = t.add2(x, const2(t, cs[-2]))
            cs = cs[:-2]
        else:
            acc = const2(t, cs[-1])
            cs = cs[:-1]
        for cf in reversed(cs):
            acc = t.add2(t.mat2(t.mul2(acc, x)), const2(t, cf))
        return t.mat2(acc)

    xn = horner(xnum, False)
    xd = horner(xden, True)
    yn = horner(ynum, False)
    yd = horner(yden, True)
    t.c.zcheck(xd[0])
    t.c.zcheck(xd[1])
    t.c.zcheck(yd[0])
    t.c.zcheck(yd[1])
    xd2 = t.mat2(t.sqr2(xd))
    yd2 = t.mat2(t.sqr2(yd))
    Z = t.mat2(t.mul2(xd, yd))
    X = t.mat2(t.mul2(xn, t.mat2(t.mul2(xd, yd2))))
    Y = t.mat2(t.mul2(t.mat2(t.mul2(y, yn)), t.mat2(t.mul2(t.mat2(t.mul2(xd, xd2)), yd2))))
    return X, Y, Z


def const2(t, v):
    return (t.c.const(v[0]) if v[0] else Lin(), t.c.const(v[1]) if v[1] else Lin())


SET_SLOTS = 92   # registers per set; packed set s uses slots [s * SET_SLOTS, (s + 1) * SET_SLOTS)


def build_pset(consts, T, miller_dbl, miller_add, X_ABS, FRAME, PSI, ISO, S=1, prefix="pset"):
    """The per-set programs for S sets packed in one wavefront (set s at register
    offset s * SET_SLOTS; its zero-checks carry its set index).  The programs carry the
    |x| chains only: RG = [s] g1 and RP = [s] pk come from k_pre's GLV lanes, loaded into
    the frame with the set's inputs."""
    progs = []
    offs = [SET_SLOTS * s for s in range(S)]
    regs = set(range(0, SET_SLOTS * S))

    def new(name):
        c = Circuit(f"{prefix}_{name}", consts)
        t = T(c)
        return c, t, F1(c), F2(t)

    def per_set(c, body):
        for s, o in enumerate(offs):
            c.zset = s
            body(o)
        c.zset = 0

    # P = iso(q0) + iso(q1); initialise every chain
    c, t, f1, f2 = new("prep")

    def prep(o):
        p0 = iso_jac(t, t.f2(o + Q0), t.f2(o + Q0 + 2), ISO)
        p1 = iso_jac(t, t.f2(o + Q1), t.f2(o + Q1 + 2), ISO)
        pp = add_gen(f2, p0, p1)
        out_jac(f2, o + PP, pp)
        out_jac(f2, o + A, pp)
        sig = aff(f2, o + SIG)
        sigj = (sig[0], sig[1], f2.one())
        out_jac(f2, o + C, sigj)

    per_set(c, prep)
    progs.append(schedule(c, FRAME, regs))

    # doubling programs
    def dbl_prog(name, g2_regs, g1_regs):
        c, t, f1, f2 = new(name)

        def body(o):
            for base in g2_regs:
                out_jac(f2, o + base, dbl(f2, jac(f2, o + base)))
            for base in g1_regs:
                out_jac(f1, o + base, dbl(f1, jac(f1, o + base)))

        per_set(c, body)
        progs.append(schedule(c, FRAME, regs))

    dbl_prog("dbl_all", (A, C), ())

    # addition at a set bit of |x|
    c, t, f1, f2 = new("add_x")

    def add_x(o):
        out_jac(f2, o + A, add_gen(f2, jac(f2, o + A), jac(f2, o + PP)))
        out_jac(f2, o + C, add_mixed(f2, jac(f2, o + C), aff(f2, o + SIG)))

    per_set(c, add_x)
    progs.append(schedule(c, FRAME, regs))

    # phase 2 (straight line): finish the cofactor clearing, the r multiples and the
    # subgroup comparison
    c, t, f1, f2 = new("phase2")

    def phase2(o):
        P = jac(f2, o + PP)
        t1 = neg_pt(f2, jac(f2, o + A))                    # [x]P = -[|x|]P
        t2 = psi_jac(t, P, PSI)
        t2p = add_gen(f2, t1, t2)                          # t1 + t2
        # U = [|x|] t2p
        U = t2p
        for i in range(62, -1, -1):
            U = dbl(f2, U)
            if (X_ABS >> i) & 1:
                U = add_gen(f2, U, t2p)
        p2 = dbl(f2, P)
        t3 = psi_jac(t, psi_jac(t, p2, PSI), PSI)          # psi^2(2P)
        t3 = add_gen(f2, t3, neg_pt(f2, t2))               # - t2
        t3 = add_gen(f2, t3, neg_pt(f2, U))                # + [x] t2p
        t3 = add_gen(f2, t3, neg_pt(f2, t1))               # - t1
        hh = add_gen(f2, t3, neg_pt(f2, P))                # - P
        out_jac(f2, o + H, hh)
        # subgroup: psi(sig) == -C (= [x] sig): (psi.x) Z^2 == X and (psi.y) Z^3 == -Y
        X, Y, Z = jac(f2, o + C)
        f2.zero(Z)                                         # [|x|] sig hit infinity: exact path
        sx = t.mulc2(t.conj2(t.f2(o + SIG)), PSI[0])
        sy = t.mulc2(t.conj2(t.f2(o + SIG + 2)), PSI[1])
        z2 = t.mat2(t.sqr2(Z))
        z3 = t.mat2(t.mul2(z2, Z))
        d0 = t.sub2(t.mul2(t.mat2(sx), z2), X)
        d1 = t.add2(t.mul2(t.mat2(sy), z3), Y)
        f2.out(o + DIFF, d0)
        f2.out(o + DIFF + 2, d1)

    per_set(c, phase2)
    progs.append(schedule(c, FRAME, regs))

    # one inversion per set (H to affine): INV_IN = N(H.z)
    c, t, f1, f2 = new("norm2")

    def norm2(o):
        hz = t.f2(o + H + 4)
        nh = c.mat(c.mul(hz[0], hz[0]) + c.mul(hz[1], hz[1]))
        c.zcheck(nh)                                       # H at infinity: exact path
        c.out(o + INV_IN, nh)

    per_set(c, norm2)
    progs.append(schedule(c, FRAME, regs))

    c, t, f1, f2 = new("affine2")

    def affine2(o):
        w = Circuit.inp(o + INV_OUT)                       # 1/N(H.z)
        z = t.f2(o + H + 4)
        zi = t.mat2((c.mul(z[0], w), -c.mul(z[1], w)))
        zi2 = t.mat2(t.sqr2(zi))
        zi3 = t.mat2(t.mul2(zi2, zi))
        f2.out(o + HQ, t.mul2(t.f2(o + H), zi2))
        f2.out(o + HQ + 2, t.mul2(t.f2(o + H + 2), zi3))

    per_set(c, affine2)
    progs.append(schedule(c, FRAME, regs))

    # f = ML(RP, HQ) * ML(-RG, SIG): two-pair Miller loop sharing the squarings
    c, t, f1, f2 = new("ml2")

    def ml2(o):
        pairs = []
        for qb, pb, sgn in ((HQ, RP, 1), (SIG, RG, -1)):
            X, Y, Z = (Circuit.inp(o + pb + k) for k in range(3))
            pz3 = c.mat(c.mul(c.mat(c.mul(Z, Z)), Z))
            pxz = c.mat(c.mul(X, Z))
            pairs.append((t.f2(o + qb), t.f2(o + qb + 2), pxz, Y * sgn, pz3))
        f = miller_loop_multi(t, pairs, miller_dbl, miller_add, X_ABS)
        for k in range(2):
            for j in range(3):
                for i in range(2):
                    c.out(o + F + 6 * k + 2 * j + i, f[k][j][i])

    per_set(c, ml2)
    # last program: only its inputs are live
    live = set()
    for o in offs:
        live |= set(range(o + RP, o + RP + 3)) | set(range(o + RG, o + RG + 3)) | set(range(o + HQ, o + HQ + 4))
        live |= set(range(o + SIG, o + SIG + 4))
    progs.append(schedule(c, FRAME, live))
    return progs


def miller_loop_multi(t, pairs, miller_dbl, miller_add, X_ABS):
    """prod_k f_{|x|,Q_k}(P_k), conjugated.  Per iteration the pairs' sparse lines are
    multiplied together (in parallel with f^2) and folded into f with one Fp12 product."""
    c = t.c
    Ts = [(qx, qy, (c.one(), Lin())) for qx, qy, _, _, _ in pairs]
    f = None
    z = (Lin(), Lin())

    def line(coefs, pxz, py, pz3):
        l0, l2, l3 = coefs
        if pz3 is not None:
            l0 = t.mulfp2(l0, pz3)
        l2 = t.mulfp2(l2, pxz)
        l3 = t.mulfp2(l3, py)
        return t.mat2(l0), t.mat2(l2), t.mat2(l3)

    def lines_product(ls):
        (a0, a2, a3), (b0, b2, b3) = ls
        p00 = t.mul2(a0, b0)
        p22 = t.mul2(a2, b2)
        p33 = t.mul2(a3, b3)
        c2 = t.sub2(t.sub2(t.mul2(t.add2(a0, a2), t.add2(b0, b2)), p00), p22)
        c3 = t.sub2(t.sub2(t.mul2(t.add2(a0, a3), t.add2(b0, b3)), p00), p33)
        c5 = t.sub2(t.sub2(t.mul2(t.add2(a2, a3), t.add2(b2, b3)), p22), p33)
        c0 = t.add2(p00, t.xi2(p33))
        return t.mat12(t.from_coefs([c0, z, c2, c3, p22, c5]))

    def step(f, ls):
        if len(ls) == 1:
            l0, l2, l3 = ls[0]
            if f is None:
                return ((l0, l2, z), (z, l3, z))
            return t.mat12(t.mul_line(f, l0, l2, l3))
        # lines two by two (sparse x sparse), then a product tree of the results
        Ls = [lines_product(ls[k:k + 2]) for k in range(0, len(ls), 2)]
        while len(Ls) > 1:
            Ls = [t.mat12(t.mul12(Ls[k], Ls[k + 1])) if k + 1 < len(Ls) else Ls[k] for k in range(0, len(Ls), 2)]
        L = Ls[0]
        return L if f is None else t.mat12(t.mul12(f, L))

    for i in range(62, -1, -1):
        if f is not None:
            f = t.mat12(t.sqr12(f))
        ls = []
        for k, (qx, qy, pxz, py, pz3) in enumerate(pairs):
            Tk, coefs = miller_dbl(t, *Ts[k])
            Ts[k] = tuple(t.mat2(x) for x in Tk)
            ls.append(line(coefs, pxz, py, pz3))
        f = step(f, ls)
        if (X_ABS >> i) & 1:
            ls = []
            for k, (qx, qy, pxz, py, pz3) in enumerate(pairs):
                Tk, coefs = miller_add(t, *Ts[k], qx, qy)
                Ts[k] = tuple(t.mat2(x) for x in Tk)
                ls.append(line(coefs, pxz, py, pz3))
            f = step(f, ls)
    return t.conj12(f)


def run_pset(pg, consts, frame, rg, rp, simulate, inv):
    """The k_pset controller (lodestar_amd/csrc/kernels/k_pset.hip) over the
    simulator: returns the zero-check flag and the subgroup result.  rg, rp: [s] g1 and
    [s] pk as G1 Jacobian triples (k_pre's GLV lanes; the kernel loads them into the
    frame with the set's inputs); pg: name -> Program; inv: Fp inverse."""
    frame[RG:RG + 3] = list(rg)
    frame[RP:RP + 3] = list(rp)
    flag = simulate(pg["pset_prep"], frame, consts)
    for i in range(62, -1, -1):
        flag |= simulate(pg["pset_dbl_all"], frame, consts)
        if (X_ABS_BITS >> i) & 1:
            flag |= simulate(pg["pset_add_x"], frame, consts)
    flag |= simulate(pg["pset_phase2"], frame, consts)
    in_group = all(frame[DIFF + k] == 0 for k in range(4))
    flag |= simulate(pg["pset_norm2"], frame, consts)
    frame[INV_OUT] = inv(frame[INV_IN])
    flag |= simulate(pg["pset_affine2"], frame, consts)
    flag |= simulate(pg["pset_ml2"], frame, consts)
    return flag, in_group


X_ABS_BITS = 0xD201000000010000


def run_psetn(pg, consts, frame, rpts, simulate, inv):
    """The k_psetn<S> controller (S = len(rpts) sets per wavefront) over the simulator:
    returns the zero-check flag bits and the per-set subgroup results.  frame: S *
    SET_SLOTS registers + temporaries; rpts: per set ([s] g1, [s] pk) as G1 Jacobian
    triples (k_pre's GLV lanes; the kernel loads them with the set's inputs)."""
    S = len(rpts)
    pre = f"pset{S}"
    for s, (rg, rp) in enumerate(rpts):
        frame[SET_SLOTS * s + RG:SET_SLOTS * s + RG + 3] = list(rg)
        frame[SET_SLOTS * s + RP:SET_SLOTS * s + RP + 3] = list(rp)
    flag = simulate(pg[f"{pre}_prep"], frame, consts)
    for i in range(62, -1, -1):
        flag |= simulate(pg[f"{pre}_dbl_all"], frame, consts)
        if (X_ABS_BITS >> i) & 1:
            flag |= simulate(pg[f"{pre}_add_x"], frame, consts)
    flag |= simulate(pg[f"{pre}_phase2"], frame, consts)
    in_group = [all(frame[SET_SLOTS * s + DIFF + k] == 0 for k in range(4)) for s in range(S)]
    flag |= simulate(pg[f"{pre}_norm2"], frame, consts)
    for s in range(S):
        frame[SET_SLOTS * s + INV_OUT] = inv(frame[SET_SLOTS * s + INV_IN])
    flag |= simulate(pg[f"{pre}_affine2"], frame, consts)
    flag |= simulate(pg[f"{pre}_ml2"], frame, consts)
    return flag, in_group


# ----------------------------------------------------------------------------
# single-pair Miller loops (k_mln after k_chain, signature pairing aggregated)
# ----------------------------------------------------------------------------
ML1_SLOTS = 19                 # per packed set: RP 0..2 (G1 Jacobian), HQ 3..6 (affine), F 7..18
ML1_RP, ML1_HQ, ML1_F = 0, 3, 7


def build_ml1(consts, T, miller_dbl, miller_add, X_ABS, FRAME, S=1, prefix="ml1"):
    """f_s = ML(RP_s, HQ_s) for S sets packed in one wavefront (set s at slot offset
    ML1_SLOTS * s): one pair per set, the signature side of the batch equation is
    summed over the group (sum r_i sig_i) and paired once per group as a further
    "set" with RP = -g1 (bls_gpu.hip, kernels/k_chain.hip)."""
    c = Circuit(f"{prefix}_{S}", consts)
    t = T(c)
    for s in range(S):
        o = ML1_SLOTS * s
        c.zset = s
        X, Y, Z = (Circuit.inp(o + ML1_RP + k) for k in range(3))
        pz3 = c.mat(c.mul(c.mat(c.mul(Z, Z)), Z))
        pxz = c.mat(c.mul(X, Z))
        f = miller_loop_multi(t, [(t.f2(o + ML1_HQ), t.f2(o + ML1_HQ + 2), pxz, Y, pz3)], miller_dbl, miller_add,
                              X_ABS)
        for k in range(2):
            for j in range(3):
                for i in range(2):
                    c.out(o + ML1_F + 6 * k + 2 * j + i, f[k][j][i])
    c.zset = 0
    live = set()
    for s in range(S):
        o = ML1_SLOTS * s
        live |= set(range(o, o + ML1_F))
    return schedule(c, FRAME, live)
