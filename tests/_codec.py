"""Byte <-> oracle-object conversions shared by the tests (canonical big-endian)."""
from __future__ import annotations

from oracle import bls_oracle as O

P = O.P


def b48(v: int) -> bytes:
    return v.to_bytes(48, "big")


def fp(b: bytes) -> int:
    return int.from_bytes(b, "big")


def f2b(x) -> bytes:
    return b48(x[0]) + b48(x[1])


def bf2(b: bytes):
    return (fp(b[:48]), fp(b[48:96]))


def f12b(f) -> bytes:
    return b"".join(f2b(c) for c in f)


def bf12(b: bytes):
    return [bf2(b[96 * k: 96 * k + 96]) for k in range(6)]


def g1b(p) -> bytes:
    return O.g1_serialize(p)


def bg1(b: bytes):
    if b[0] & 0x40:
        return None
    return (fp(b[:48]), fp(b[48:96]))


def g2b(p) -> bytes:
    if p is None:
        return bytes([0x40]) + bytes(191)
    (x0, x1), (y0, y1) = p
    return b48(x1) + b48(x0) + b48(y1) + b48(y0)


def bg2(b: bytes):
    if b[0] & 0x40:
        return None
    return ((fp(b[48:96]), fp(b[0:48])), (fp(b[144:192]), fp(b[96:144])))


def sk_bytes(sk: int) -> bytes:
    return sk.to_bytes(32, "big")
