"""bls/lazy28.hpp (14 x 28-bit digits, Montgomery R' = 2^392, bounds in the type) compiled
for the CPU (tests/native/hostsim.cpp) against Python big integers: the raw product at
the edges of its digit bounds, every additive operation, the conversions, and the Fp2
tower -- bit-exact after conversion back to canonical Fp."""
from __future__ import annotations

import ctypes
import random

from tests._codec import P, b48, fp

M28 = (1 << 28) - 1
RP_INV = pow(2, -392, P)


def _val(d) -> int:
    return sum(int(x) << (28 * k) for k, x in enumerate(d))


def _arr(d):
    return (ctypes.c_int32 * 14)(*d)


def _signed_digits(v: int, rng, dmax: int) -> list[int]:
    """A signed digit vector of value v (any sign) with |digits| pushed up to dmax (moving
    multiples of 2^28 between neighbouring digits), so the product sees unnormalised,
    mixed-sign operands."""
    d = [0] * 14
    m = abs(v)
    for k in range(13):
        d[k] = (m >> (28 * k)) & M28
    d[13] = m >> (28 * 13)
    if v < 0:
        d = [-x for x in d]
    for k in range(13):
        # move t units of digit k+1 into digit k (value unchanged)
        for _ in range(3):
            t = rng.randint(-4, 4)
            nk, nk1 = d[k] + t * (1 << 28), d[k + 1] - t
            if abs(nk) <= dmax and abs(nk1) <= dmax:
                d[k], d[k + 1] = nk, nk1
    assert _val(d) == v and max(abs(x) for x in d) <= dmax
    return d


def test_lazy28_raw_product_bounds(hostsim):
    """lz_mul_core / lz_sqr_core on signed digits: x y / 2^392 mod p, digits 0..12 of the
    output in [0, 2^28), |value| < p + |x y| / 2^392, for operands at the largest digits
    lz_mul_fits admits (|digit| ~2^29.5 each side) and large magnitudes of either sign."""
    rng = random.Random(392)
    out = (ctypes.c_int32 * 14)()
    cases = []
    for _ in range(300):
        vx = rng.randrange(1 << rng.choice((10, 200, 381, 384, 388))) * rng.choice((1, -1))
        vy = rng.randrange(1 << rng.choice((10, 200, 381, 384, 388))) * rng.choice((1, -1))
        cases.append((vx, vy))
    cases += [(0, 0), (P - 1, P - 1), (-(2 * P - 1), 2 * P - 1), (256 * P - 1, -9 * P), ((1 << 388) - 1, P)]
    dmax = int(2 ** 29.5)
    for vx, vy in cases:
        x = _signed_digits(vx, rng, dmax)
        y = _signed_digits(vy, rng, dmax)
        for sqr in (0, 1):
            yv = vx if sqr else vy
            hostsim.hs_lz_mul_raw(_arr(x), _arr(x if sqr else y), out, sqr)
            r = list(out)
            assert all(0 <= c <= M28 for c in r[:13])
            rv = _val(r)
            assert rv % P == (vx * yv * RP_INV) % P
            assert abs(rv) < P + abs(vx * yv) // (1 << 392) + 1


def test_lazy28_fp_ops(hostsim):
    """lz_from_fp -> lazy formulas -> lz_to_fp equals the field arithmetic."""
    rng = random.Random(28)
    out = ctypes.create_string_buffer(10 * 48)
    vals = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, 2 ** 380, 2 ** 381 - 1 if 2 ** 381 - 1 < P else P - 3]
    vals += [rng.randrange(P) for _ in range(200)]
    for k, a in enumerate(vals):
        b = vals[(7 * k + 3) % len(vals)]
        hostsim.hs_lz_fp_ops(b48(a), b48(b), out)
        r = [fp(out.raw[48 * i: 48 * i + 48]) for i in range(10)]
        ab = a * b % P
        assert r[0] == ab
        assert r[1] == a * a % P
        assert r[2] == (a + b) % P
        assert r[3] == (a - b) % P
        assert r[4] == (-ab) % P
        assert r[5] == ab * pow(2, -1, P) % P
        assert r[6] == (-ab) % P
        assert r[7] == (2 * ab - b * b) * (b - a) % P
        assert r[8] == a
        assert r[9] == 4 * (2 * ab - 7 * b * b - 7 * a) % P


def test_lazy28_fp2_ops(hostsim):
    """l2_mul / l2_sqr / l2_mul_xi / l2_conj / l2_sub / l2_mul_fp against Fp2 = Fp[u]/(u^2+1)."""
    rng = random.Random(29)
    out = ctypes.create_string_buffer(6 * 96)

    def mul(x, y):
        return ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)

    edge = [0, 1, P - 1, (P - 1) // 2]
    for k in range(150):
        a = (rng.choice(edge) if k < 16 else rng.randrange(P), rng.randrange(P) if k % 3 else rng.choice(edge))
        b = (rng.randrange(P), rng.choice(edge) if k % 5 == 0 else rng.randrange(P))
        hostsim.hs_lz_fp2_ops(b48(a[0]) + b48(a[1]), b48(b[0]) + b48(b[1]), out)
        r = [(fp(out.raw[96 * i: 96 * i + 48]), fp(out.raw[96 * i + 48: 96 * i + 96])) for i in range(6)]
        m = mul(a, b)
        assert r[0] == m
        assert r[1] == mul(a, a)
        assert r[2] == ((m[0] - m[1]) % P, (m[0] + m[1]) % P)
        assert r[3] == (m[0], (-m[1]) % P)
        bb = mul(b, b)
        assert r[4] == ((m[0] - bb[0]) % P, (m[1] - bb[1]) % P)
        assert r[5] == (m[0] * b[0] % P, m[1] * b[0] % P)
