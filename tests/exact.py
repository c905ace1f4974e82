"""Exact IEEE binary32 arithmetic on rationals, for hand-derived oracle KATs.

Each helper computes the exact real result with fractions.Fraction and rounds
it ONCE to the nearest float32 (ties to even) -- the semantics of one IEEE op
(fmul, fadd) or of one fused multiply-add (ffma).
"""
from fractions import Fraction

import numpy as np


def F(x) -> Fraction:
    return Fraction(float(np.float32(x)))


def round_f32(v: Fraction) -> np.float32:
    if v == 0:
        return np.float32(0.0)
    sign = -1 if v < 0 else 1
    a = abs(v)
    e = a.numerator.bit_length() - a.denominator.bit_length()
    while Fraction(2) ** e > a:
        e -= 1
    while Fraction(2) ** (e + 1) <= a:
        e += 1
    e = max(e, -126)
    scale = Fraction(2) ** (e - 23)
    m = a / scale
    q = m.numerator // m.denominator
    rem = m - q
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and q % 2 == 1):
        q += 1
    return np.float32(sign * float(Fraction(q) * scale))


def fmul(a, b):
    return round_f32(F(a) * F(b))


def fadd(a, b):
    return round_f32(F(a) + F(b))


def fsub(a, b):
    return round_f32(F(a) - F(b))


def ffma(a, b, c):
    return round_f32(F(a) * F(b) + F(c))


def bits(x) -> int:
    return int(np.float32(x).view(np.uint32))
