"""CPU ORACLE — test infrastructure only. Never shipped, never on the product path.

Spec-level restatement of the BLS12-381 signature-verification algorithm that the
reference (Lodestar, /root/reference) reaches through its un-vendored npm dependency
chain `@chainsafe/bls@7.1.x` -> `@chainsafe/blst@0.2.4` -> supranational `blst`
(pinned at `yarn.lock:427-451`; none of it is present under /root/reference).
Because the library is absent, this module restates the *published* algorithms:

* IETF BLS signature draft, proof-of-possession ciphersuite
  `BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_` (the DST Lodestar/blst use);
* RFC 9380 (hash-to-curve) suite `BLS12381G2_XMD:SHA-256_SSWU_RO_`:
  expand_message_xmd, hash_to_field, simplified SWU on the 3-isogenous E2',
  the 3-isogeny map, clear_cofactor via h_eff;
* ZCash BLS12-381 point serialization (flag bits C/I/S in byte 0);
* optimal-ate pairing, Miller loop over |x| = 0xd201000000010000 with the result
  conjugated because x < 0, final exponentiation (p^12-1)/r.

Reference call sites this restates (file:line under /root/reference/packages):
* `beacon-node/src/chain/bls/maybeBatch.ts:16-39`  verifySignatureSetsMaybeBatch
* `beacon-node/src/chain/bls/utils.ts:5-16`        getAggregatedPubkey
* `beacon-node/src/chain/bls/multithread/worker.ts:32-108` verifyManySignatureSets
* `beacon-node/src/chain/bls/multithread/utils.ts:4-19`    chunkifyMaximizeChunkSize
* `state-transition/src/util/interop.ts:19-22`     interop secret keys (fixtures)

Pinned by the reference's own known-answer data (see tests/test_oracle_kat.py):
KAT-1 interop deposit signature (`beacon-node/test/e2e/interop/genesisState.test.ts:65-69`),
KAT-2 100 interop pubkeys (`state-transition/test-cache/interop-pubkeys.json`),
KAT-3 real mainnet G2 points (`beacon-node/test/unit/sync/backfill/blocks.json`).

Pure Python big-int arithmetic: slow (a pairing takes ~0.5 s) and meant for small
cases only.  The multi-threaded C++ restatement of the reference's worker pool that
bench.py times as the CPU baseline lives in `oracle/cpu/bls_cpu.cpp` ("not blst").
"""
from __future__ import annotations

import hashlib
import secrets

# ----------------------------------------------------------------------------
# Curve constants
# ----------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000  # |x|, x = -X_ABS is the BLS parameter
X_NEG = True
DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

# ZCash-format error strings used by the reference stack ([ext] @chainsafe/blst).
# Only the BLST_INVALID_SIZE substring and the "BLST_ERROR" prefix are pinned by
# the reference's own tests (multithread.test.ts:100, spec/general/bls.ts:37).
E_OK = 0
E_BAD_ENCODING = 1
E_POINT_NOT_ON_CURVE = 2
E_POINT_NOT_IN_GROUP = 3
E_PK_IS_INFINITY = 6
E_INVALID_SIZE = 8
E_ZERO_SIGNATURE = 9
E_EMPTY_SET = 10
E_EMPTY_AGGREGATE = 11
ERROR_NAMES = {
    E_BAD_ENCODING: "BLST_BAD_ENCODING",
    E_POINT_NOT_ON_CURVE: "BLST_POINT_NOT_ON_CURVE",
    E_POINT_NOT_IN_GROUP: "BLST_POINT_NOT_IN_GROUP",
    E_PK_IS_INFINITY: "BLST_PK_IS_INFINITY",
    E_INVALID_SIZE: "BLST_INVALID_SIZE",
}


class BlsError(Exception):
    """Mirrors the reference's error convention: message contains the BLST_* code."""

    def __init__(self, code: int):
        self.code = code
        if code in ERROR_NAMES:
            msg = "BLST_ERROR: " + ERROR_NAMES[code]
        elif code == E_ZERO_SIGNATURE:
            msg = "ZERO_SIGNATURE"
        elif code == E_EMPTY_SET:
            msg = "Empty signature set"
        elif code == E_EMPTY_AGGREGATE:
            msg = "EMPTY_AGGREGATE_ARRAY"
        else:
            msg = "BLST_ERROR: code %d" % code
        super().__init__(msg)


# ----------------------------------------------------------------------------
# Fp2 = Fp[i]/(i^2+1), elements as tuples (c0, c1)
# ----------------------------------------------------------------------------
def f2(a, b=0):
    return (a % P, b % P)


F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, s):
    return ((a[0] * s) % P, (a[1] * s) % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = pow(n, P - 2, P)
    return ((a[0] * ni) % P, (-a[1] * ni) % P)


def f2_pow(a, e):
    r = F2_ONE
    b = a
    while e:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_sqr(b)
        e >>= 1
    return r


def f2_is_zero(a):
    return a[0] == 0 and a[1] == 0


def legendre(a):
    a %= P
    if a == 0:
        return 0
    return 1 if pow(a, (P - 1) // 2, P) == 1 else -1


def f2_is_square(a):
    # a is a square in Fp2 iff its norm is a square in Fp
    return legendre(a[0] * a[0] + a[1] * a[1]) >= 0


def f2_sqrt(a):
    """Some square root of a, or None.  (Adj & Rodriguez-Henriquez, Alg. 9, p = 3 mod 4)."""
    if f2_is_zero(a):
        return F2_ZERO
    a1 = f2_pow(a, (P - 3) // 4)
    alpha = f2_mul(f2_sqr(a1), a)
    x0 = f2_mul(a1, a)
    if alpha == (P - 1, 0):
        x = f2_mul((0, 1), x0)
    else:
        b = f2_pow(f2_add(F2_ONE, alpha), (P - 1) // 2)
        x = f2_mul(b, x0)
    if f2_sqr(x) != a:
        return None
    return x


def fp_sqrt(a):
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if (s * s) % P == a else None


def sgn0_f2(a):
    """RFC 9380 sgn0 for m = 2."""
    s0 = a[0] & 1
    z0 = a[0] == 0
    s1 = a[1] & 1
    return s0 | (z0 & s1)


def lex_largest_fp(a):
    return a > (P - 1) // 2


def lex_largest_f2(a):
    # ZCash serialization sign: compare c1 first, c0 if c1 == 0
    if a[1] != 0:
        return lex_largest_fp(a[1])
    return lex_largest_fp(a[0])


# ----------------------------------------------------------------------------
# Generic short-Weierstrass y^2 = x^3 + a x + b, affine, None = infinity.
# Field ops are passed as a small table so one implementation serves E1/E2/E2'.
# ----------------------------------------------------------------------------
class FieldOps:
    def __init__(self, add, sub, mul, inv, neg, zero, one, small):
        self.add, self.sub, self.mul, self.inv, self.neg = add, sub, mul, inv, neg
        self.zero, self.one, self.small = zero, one, small


FP_OPS = FieldOps(
    lambda a, b: (a + b) % P,
    lambda a, b: (a - b) % P,
    lambda a, b: (a * b) % P,
    lambda a: pow(a, P - 2, P),
    lambda a: (-a) % P,
    0,
    1,
    lambda k: k % P,
)
FP2_OPS = FieldOps(f2_add, f2_sub, f2_mul, f2_inv, f2_neg, F2_ZERO, F2_ONE, lambda k: (k % P, 0))


class Curve:
    def __init__(self, F: FieldOps, a, b):
        self.F, self.a, self.b = F, a, b

    def on_curve(self, pt):
        if pt is None:
            return True
        F = self.F
        x, y = pt
        lhs = F.mul(y, y)
        rhs = F.add(F.add(F.mul(F.mul(x, x), x), F.mul(self.a, x)), self.b)
        return lhs == rhs

    def neg(self, pt):
        if pt is None:
            return None
        return (pt[0], self.F.neg(pt[1]))

    def add(self, p1, p2):
        F = self.F
        if p1 is None:
            return p2
        if p2 is None:
            return p1
        x1, y1 = p1
        x2, y2 = p2
        if x1 == x2:
            if y1 == y2 and y1 != F.zero:
                # doubling
                num = F.add(F.mul(F.small(3), F.mul(x1, x1)), self.a)
                lam = F.mul(num, F.inv(F.add(y1, y1)))
            else:
                return None
        else:
            lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
        x3 = F.sub(F.sub(F.mul(lam, lam), x1), x2)
        y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
        return (x3, y3)

    def dbl(self, p):
        return self.add(p, p)

    def mul(self, pt, k):
        if k < 0:
            return self.mul(self.neg(pt), -k)
        acc = None
        base = pt
        while k:
            if k & 1:
                acc = self.add(acc, base)
            base = self.dbl(base)
            k >>= 1
        return acc


B2 = (4, 4)  # 4(1+i)
E1 = Curve(FP_OPS, 0, 4)
E2 = Curve(FP2_OPS, F2_ZERO, B2)
# E2': y^2 = x^3 + 240 i x + 1012 (1 + i)
A_ISO = (0, 240)
B_ISO = (1012, 1012)
E2_ISO = Curve(FP2_OPS, A_ISO, B_ISO)
Z_SSWU = f2(-2, -1)

G1 = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2 = (
    (
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    (
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)

# ----------------------------------------------------------------------------
# Serialization (ZCash format)
# ----------------------------------------------------------------------------
def i2b(v, n):
    return v.to_bytes(n, "big")


def g1_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    b = bytearray(i2b(x, 48))
    b[0] |= 0x80
    if lex_largest_fp(y):
        b[0] |= 0x20
    return bytes(b)


def g1_serialize(pt):
    """96-byte uncompressed form (what the reference pool sends to workers, index.ts:126,160)."""
    if pt is None:
        return bytes([0x40]) + bytes(95)
    return i2b(pt[0], 48) + i2b(pt[1], 48)


def g1_decompress(b: bytes):
    """Returns (code, point).  No subgroup check (reference keys are trusted)."""
    if len(b) != 48:
        return E_INVALID_SIZE, None
    c, inf, s = b[0] >> 7 & 1, b[0] >> 6 & 1, b[0] >> 5 & 1
    if not c:
        return E_BAD_ENCODING, None
    if inf:
        if (b[0] & 0x3F) == 0 and not any(b[1:]):
            return E_OK, None
        return E_BAD_ENCODING, None
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big")
    if x >= P:
        return E_BAD_ENCODING, None
    y = fp_sqrt(x * x * x + 4)
    if y is None:
        return E_POINT_NOT_ON_CURVE, None
    if lex_largest_fp(y) != bool(s):
        y = (-y) % P
    return E_OK, (x, y)


def g1_deserialize(b: bytes):
    """96-byte uncompressed G1 (blst_p1_deserialize semantics, on-curve check only)."""
    if len(b) != 96:
        return E_INVALID_SIZE, None
    if b[0] & 0x80:
        return E_BAD_ENCODING, None
    if b[0] & 0x40:
        if (b[0] & 0x3F) == 0 and not any(b[1:]):
            return E_OK, None
        return E_BAD_ENCODING, None
    if b[0] & 0x20:
        return E_BAD_ENCODING, None
    x = int.from_bytes(b[:48], "big")
    y = int.from_bytes(b[48:], "big")
    if x >= P or y >= P:
        return E_BAD_ENCODING, None
    if not E1.on_curve((x, y)):
        return E_POINT_NOT_ON_CURVE, None
    return E_OK, (x, y)


def g2_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    b = bytearray(i2b(x[1], 48) + i2b(x[0], 48))
    b[0] |= 0x80
    if lex_largest_f2(y):
        b[0] |= 0x20
    return bytes(b)


def g2_decompress(b: bytes):
    """blst_p2_uncompress semantics: returns (code, point); no subgroup check here."""
    if len(b) != 96:
        return E_INVALID_SIZE, None
    c, inf, s = b[0] >> 7 & 1, b[0] >> 6 & 1, b[0] >> 5 & 1
    if not c:
        return E_BAD_ENCODING, None
    if inf:
        if (b[0] & 0x3F) == 0 and not any(b[1:]):
            return E_OK, None
        return E_BAD_ENCODING, None
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x1 >= P or x0 >= P:
        return E_BAD_ENCODING, None
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        return E_POINT_NOT_ON_CURVE, None
    if lex_largest_f2(y) != bool(s):
        y = f2_neg(y)
    return E_OK, (x, y)


def g2_in_subgroup(pt):
    """Naive r*P == O membership test (GPU uses psi(P) == [x]P; the two must agree)."""
    return E2.mul(pt, R) is None


def g1_in_subgroup(pt):
    """Naive r*P == O membership test (GPU uses sigma(P) == [-x^2]P; the two must agree)."""
    return E1.mul(pt, R) is None


def key_validate(b: bytes) -> int:
    """blst PublicKey.fromBytes(b, validate=true) [ext] as the deposit path uses it
    (state-transition block/processDeposit.ts:56-65): decode (48 compressed or 96
    uncompressed), infinity -> BLST_PK_IS_INFINITY, outside G1 -> BLST_POINT_NOT_IN_GROUP.
    Returns 0 or the error code."""
    code, pt = g1_decompress(b) if len(b) == 48 else g1_deserialize(b)
    if code != E_OK:
        return code
    if pt is None:
        return E_PK_IS_INFINITY
    return E_OK if g1_in_subgroup(pt) else E_POINT_NOT_IN_GROUP


def signature_from_bytes(b: bytes, validate=True):
    """Signature.fromBytes(b, affine, validate) [ext]: decode + optional subgroup check."""
    code, pt = g2_decompress(b)
    if code != E_OK:
        raise BlsError(code)
    if validate and pt is not None and not g2_in_subgroup(pt):
        raise BlsError(E_POINT_NOT_IN_GROUP)
    return pt


# ----------------------------------------------------------------------------
# hash_to_G2 (RFC 9380, BLS12381G2_XMD:SHA-256_SSWU_RO_)
# ----------------------------------------------------------------------------
def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    b_in_bytes, r_in_bytes = 32, 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(r_in_bytes)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, count: int, dst: bytes):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    us = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(ub[off : off + L], "big") % P)
        us.append((e[0], e[1]))
    return us


def map_to_curve_sswu(u):
    """Simplified SWU onto E2' (RFC 9380 6.6.2, straightforward form)."""
    A, B, Z = A_ISO, B_ISO, Z_SSWU
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    den = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(den):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        tv1 = f2_inv(den)
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, tv1))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x = f2_mul(zu2, x1)
        gx2 = f2_add(f2_add(f2_mul(f2_sqr(x), x), f2_mul(A, x)), B)
        y = f2_sqrt(gx2)
    assert y is not None
    if sgn0_f2(u) != sgn0_f2(y):
        y = f2_neg(y)
    return (x, y)


# 3-isogeny E2' -> E2 constants (RFC 9380 Appendix E.3)
_KP = P
ISO_XNUM = [
    (0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
     0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    (0, 0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    (0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
]
ISO_XDEN = [
    (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63),
    (0xC, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F),
    (1, 0),
]
ISO_YNUM = [
    (0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
     0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    (0, 0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    (0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
]
ISO_YDEN = [
    (0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
     0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB),
    (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3),
    (0x12, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99),
    (1, 0),
]


def _poly(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map(pt):
    if pt is None:
        return None
    x, y = pt
    xn, xd = _poly(ISO_XNUM, x), _poly(ISO_XDEN, x)
    yn, yd = _poly(ISO_YNUM, x), _poly(ISO_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    return (f2_mul(xn, f2_inv(xd)), f2_mul(y, f2_mul(yn, f2_inv(yd))))


# psi endomorphism: psi(x, y) = (conj(x) * PSI_X, conj(y) * PSI_Y)
_XI = (1, 1)
PSI_X = f2_inv(f2_pow(_XI, (P - 1) // 3))
PSI_Y = f2_inv(f2_pow(_XI, (P - 1) // 2))


def psi(pt):
    if pt is None:
        return None
    return (f2_mul(f2_conj(pt[0]), PSI_X), f2_mul(f2_conj(pt[1]), PSI_Y))


H_EFF = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551
X_PARAM = -X_ABS


def clear_cofactor_g2(pt):
    """RFC 9380 Appendix G.3 (Budroni-Pintore), equal to [h_eff]P."""
    t1 = E2.mul(pt, X_PARAM)
    t2 = psi(pt)
    t3 = E2.dbl(pt)
    t3 = psi(psi(t3))
    t3 = E2.add(t3, E2.neg(t2))
    t2 = E2.add(t1, t2)
    t2 = E2.mul(t2, X_PARAM)
    t3 = E2.add(t3, t2)
    t3 = E2.add(t3, E2.neg(t1))
    return E2.add(t3, E2.neg(pt))


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = iso_map(map_to_curve_sswu(u0))
    q1 = iso_map(map_to_curve_sswu(u1))
    return clear_cofactor_g2(E2.add(q0, q1))


# ----------------------------------------------------------------------------
# Fp12 = Fp2[w]/(w^6 - xi), xi = 1 + i.  Element: list of 6 Fp2 coefficients.
# (Same basis as the GPU tower: Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v),
#  coefficient k of w^k <-> (a0,b0,a1,b1,a2,b2).)
# ----------------------------------------------------------------------------
F12_ONE = [F2_ONE] + [F2_ZERO] * 5


def f12_mul(a, b):
    t = [F2_ZERO] * 11
    for i in range(6):
        if f2_is_zero(a[i]):
            continue
        for j in range(6):
            if f2_is_zero(b[j]):
                continue
            t[i + j] = f2_add(t[i + j], f2_mul(a[i], b[j]))
    out = t[:6]
    for k in range(6, 11):
        out[k - 6] = f2_add(out[k - 6], f2_mul(t[k], _XI))
    return out


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    # a^(p^6): w -> -w
    return [c if k % 2 == 0 else f2_neg(c) for k, c in enumerate(a)]


def f12_pow(a, e):
    r = F12_ONE
    b = a
    while e:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_sqr(b)
        e >>= 1
    return r


def f12_frob(a):
    # a^p: coefficient k -> conj(c_k) * xi^((p-1)k/6)
    return [f2_mul(f2_conj(c), f2_pow(_XI, (P - 1) * k // 6)) for k, c in enumerate(a)]


def f12_inv(a):
    # a^-1 = a^(p^12 - 2) is slow; use norm to Fp6 via conj: a * conj(a) in Fp6 (even coeffs)
    # Fall back to the generic exponent for simplicity (oracle only, rare use).
    return f12_pow(a, P**12 - 2)


def f12_is_one(a):
    return a == F12_ONE


# Line evaluation with the untwisted point.  Q' = (x', y') on E2 (M-twist) maps to
# E(Fp12) as (x' / w^2, y' / w^3).  We keep everything in the w-basis.
def _f12_from_f2_at(c, k):
    v = [F2_ZERO] * 6
    v[k] = c
    return v


_W_INV = [F2_ZERO] * 5 + [f2_inv(_XI)]  # w^-1 = w^5 / xi


def _untwist(Q):
    x, y = Q
    winv2 = f12_mul(_W_INV, _W_INV)
    winv3 = f12_mul(winv2, _W_INV)
    return (f12_mul(_f12_from_f2_at(x, 0), winv2), f12_mul(_f12_from_f2_at(y, 0), winv3))


def _f12_sub(a, b):
    return [f2_sub(x, y) for x, y in zip(a, b)]


def _f12_add(a, b):
    return [f2_add(x, y) for x, y in zip(a, b)]


def _f12_scalar(s):
    return [(s % P, 0)] + [F2_ZERO] * 5


def _f12_inv_slow(a):
    return f12_inv(a)


def miller_loop(Pp, Qp):
    """Optimal-ate Miller loop f_{|x|,Q}(P), conjugated since x < 0.  Textbook affine form
    in Fp12 (vertical lines dropped: they lie in a subfield killed by the final exponentiation).
    Returns F12_ONE if either point is infinity."""
    if Pp is None or Qp is None:
        return F12_ONE
    Qx, Qy = _untwist(Qp)
    Px, Py = _f12_scalar(Pp[0]), _f12_scalar(Pp[1])
    Tx, Ty = Qx, Qy
    f = F12_ONE
    bits = bin(X_ABS)[3:]
    inv = _f12_inv_fast
    for bit in bits:
        # doubling: lambda = 3 x^2 / 2 y
        lam = f12_mul(f12_mul(_f12_scalar(3), f12_sqr(Tx)), inv(_f12_add(Ty, Ty)))
        line = _f12_sub(_f12_sub(Py, Ty), f12_mul(lam, _f12_sub(Px, Tx)))
        f = f12_mul(f12_sqr(f), line)
        nx = _f12_sub(_f12_sub(f12_sqr(lam), Tx), Tx)
        ny = _f12_sub(f12_mul(lam, _f12_sub(Tx, nx)), Ty)
        Tx, Ty = nx, ny
        if bit == "1":
            lam = f12_mul(_f12_sub(Qy, Ty), inv(_f12_sub(Qx, Tx)))
            line = _f12_sub(_f12_sub(Py, Ty), f12_mul(lam, _f12_sub(Px, Tx)))
            f = f12_mul(f, line)
            nx = _f12_sub(_f12_sub(f12_sqr(lam), Tx), Qx)
            ny = _f12_sub(f12_mul(lam, _f12_sub(Tx, nx)), Ty)
            Tx, Ty = nx, ny
    if X_NEG:
        f = f12_conj(f)
    return f


def _f6_mul(a, b):
    # Fp6 = Fp2[v]/(v^3 - xi); elements as 3-lists
    t = [F2_ZERO] * 5
    for i in range(3):
        for j in range(3):
            t[i + j] = f2_add(t[i + j], f2_mul(a[i], b[j]))
    return [f2_add(t[0], f2_mul(t[3], _XI)), f2_add(t[1], f2_mul(t[4], _XI)), t[2]]


def _f6_inv(a):
    a0, a1, a2 = a
    t0 = f2_sub(f2_sqr(a0), f2_mul(_XI, f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul(_XI, f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    n = f2_add(f2_mul(a0, t0), f2_mul(_XI, f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    ni = f2_inv(n)
    return [f2_mul(t0, ni), f2_mul(t1, ni), f2_mul(t2, ni)]


def _f12_inv_fast(a):
    # a = A + B w with A = (c0, c2, c4), B = (c1, c3, c5); w^2 = v
    A = [a[0], a[2], a[4]]
    B = [a[1], a[3], a[5]]
    # (A + B w)^-1 = (A - B w) / (A^2 - B^2 v)
    A2 = _f6_mul(A, A)
    B2v = _f6_mul(B, B)
    B2v = [f2_mul(B2v[2], _XI), B2v[0], B2v[1]]  # times v
    n = [f2_sub(x, y) for x, y in zip(A2, B2v)]
    ni = _f6_inv(n)
    Ai = _f6_mul(A, ni)
    Bi = [f2_neg(c) for c in _f6_mul(B, ni)]
    return [Ai[0], Bi[0], Ai[1], Bi[1], Ai[2], Bi[2]]


f12_inv = _f12_inv_fast  # noqa: F811  (fast exact inverse)

FE_EASY = (P**6 - 1) * (P**2 + 1)
FE_HARD = (P**4 - P**2 + 1) // R
assert (P**4 - P**2 + 1) % R == 0


def final_exponentiation(f, hard_multiple=1):
    """f^((p^12-1)/r) (times `hard_multiple` in the hard part; the GPU computes 3x)."""
    # easy part: f^(p^6-1)(p^2+1)
    t = f12_mul(f12_conj(f), f12_inv(f))
    t = f12_mul(f12_frob(f12_frob(t)), t)
    return f12_pow(t, FE_HARD * hard_multiple)


def pairing(Pp, Qp):
    return final_exponentiation(miller_loop(Pp, Qp))


# ----------------------------------------------------------------------------
# Keys, signing, verification
# ----------------------------------------------------------------------------
def interop_secret_key(index: int) -> int:
    """state-transition/src/util/interop.ts:19-22: LE(sha256(LE32(i))) mod r (bytesToBigInt is LE)."""
    d = hashlib.sha256(index.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R


def sk_to_pk(sk: int):
    return E1.mul(G1, sk)


def sign(sk: int, msg: bytes, dst: bytes = DST_POP):
    return E2.mul(hash_to_g2(msg, dst), sk)


def aggregate_pubkeys(pks):
    """bls.PublicKey.aggregate (utils.ts:11): plain G1 sum; [] -> EMPTY_AGGREGATE_ARRAY."""
    if len(pks) == 0:
        raise BlsError(E_EMPTY_AGGREGATE)
    acc = None
    for pk in pks:
        acc = E1.add(acc, pk)
    return acc


def core_verify(pk, msg: bytes, sig_bytes: bytes) -> bool:
    """maybeBatch.ts:33-38 single-set path: fromBytes(sig, affine, true).verify(pk, msg).

    [ext] @chainsafe/bls Signature.verify rejects an infinity signature with ZERO_SIGNATURE;
    blst rejects an infinity public key with BLST_PK_IS_INFINITY.  (parity unpinned)"""
    sig = signature_from_bytes(sig_bytes, validate=True)
    if sig is None:
        raise BlsError(E_ZERO_SIGNATURE)
    if pk is None:
        raise BlsError(E_PK_IS_INFINITY)
    f = f12_mul(miller_loop(pk, hash_to_g2(msg)), miller_loop(E1.neg(G1), sig))
    return f12_is_one(final_exponentiation(f))


def verify_multiple(sets, scalars=None) -> bool:
    """maybeBatch.ts:18-25: Signature.verifyMultipleSignatures with validate=true.
    sets: list of (pk_point, msg, sig_bytes).  Random non-zero 64-bit scalars
    ([ext] @chainsafe/blst randomBytesNonZero(8) + blst mul_n_aggregate)."""
    sigs = [signature_from_bytes(s[2], validate=True) for s in sets]
    if scalars is None:
        scalars = [secrets.randbits(64) | 1 for _ in sets]
    f = F12_ONE
    agg = None
    for (pk, msg, _), sig, r in zip(sets, sigs, scalars):
        if pk is None:
            raise BlsError(E_PK_IS_INFINITY)
        f = f12_mul(f, miller_loop(E1.mul(pk, r), hash_to_g2(msg)))
        agg = E2.add(agg, E2.mul(sig, r)) if sig is not None else agg
    f = f12_mul(f, miller_loop(E1.neg(G1), agg))
    return f12_is_one(final_exponentiation(f))


def verify_signature_sets_maybe_batch(sets, scalars=None) -> bool:
    """maybeBatch.ts:16-39."""
    if len(sets) >= 2:
        return verify_multiple(sets, scalars)
    if len(sets) == 0:
        raise BlsError(E_EMPTY_SET)
    pk, msg, sig = sets[0]
    return core_verify(pk, msg, sig)


def chunkify_maximize_chunk_size(arr, min_per_chunk):
    """multithread/utils.ts:4-19."""
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [list(arr)]
    per_chunk = -(-len(arr) // chunk_count)
    return [list(arr[i : i + per_chunk]) for i in range(0, len(arr), per_chunk)]


def deserialize_set(s):
    """worker.ts:110-116 deserializeSet: PublicKey.fromBytes(96 B, affine), no validation.
    A set whose pubkey is already a point (or None = infinity) passes through; raw bytes
    that do not decode raise BlsError."""
    pk, msg, sig = s
    if isinstance(pk, (bytes, bytearray)):
        code, pt = g1_deserialize(bytes(pk))
        if code != E_OK:
            raise BlsError(code)
        pk = pt
    return (pk, msg, sig)


def verify_many_signature_sets(work_reqs, maybe_batch=None):
    """multithread/worker.ts:32-108.  work_reqs: list of (batchable, sets).  Returns a list of
    ("success", bool) or ("error", BlsError) per request, plus (batchRetries, batchSigsSuccess).

    deserializeSet runs over every request before any verification and outside any try
    (worker.ts:43-46): one raw pubkey that does not decode throws out of the worker call,
    and the pool rejects every job of that message with the error (index.ts:367-374) --
    so every request gets ("error", e) and the counters are meaningless (0, 0).

    maybe_batch: the crypto predicate verifySignatureSetsMaybeBatch (maybeBatch.ts:16-39)
    over a list of sets, default this module's.  Parity tests at BASELINE sizes pass one
    that reads each set's validity known by construction (the sets are then opaque
    tokens and deserializeSet is skipped), so the worker's chunking, fallback and
    bookkeeping rules below still decide the expected verdicts and counters."""
    results = [None] * len(work_reqs)
    batch_retries = 0
    batch_sigs_success = 0
    batchable, non_batchable = [], []
    if maybe_batch is None:
        maybe_batch = verify_signature_sets_maybe_batch
        try:
            work_reqs = [(b, [deserialize_set(s) for s in sets]) for b, sets in work_reqs]
        except BlsError as e:
            return [("error", e)] * len(results), 0, 0
    for i, (is_batchable, sets) in enumerate(work_reqs):
        (batchable if is_batchable else non_batchable).append((i, sets))
    if batchable:
        for chunk in chunkify_maximize_chunk_size(batchable, 16):
            all_sets = [s for _, sets in chunk for s in sets]
            try:
                ok = maybe_batch(all_sets)
            except BlsError:
                ok = None
            if ok:
                for idx, sets in chunk:
                    batch_sigs_success += len(sets)
                    results[idx] = ("success", True)
            else:
                batch_retries += 1
                non_batchable.extend(chunk)
    for idx, sets in non_batchable:
        try:
            results[idx] = ("success", maybe_batch(sets))
        except BlsError as e:
            results[idx] = ("error", e)
    return results, batch_retries, batch_sigs_success
