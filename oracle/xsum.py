"""Test infrastructure: restatement of the engine's order-independent CG sums
(movie_recommender_amd/csrc/kernels.hip ``xterm`` / ``xsum_value``): every
term truncated toward zero to a multiple of 2^-192 and summed exactly as an
integer; the integer is cut into ten 32-bit digits (the top one signed) and
converted by Horner's rule in base 2^32 in IEEE double arithmetic, then
scaled by 2^-192.  A term that is not finite or has |t| >= 2^96 makes the
sum NaN.  The device result must equal this bit for bit."""
import math
from fractions import Fraction

XD, LSB = 10, -192


def xsum(terms):
    total = 0
    for t in terms:
        t = float(t)
        if not math.isfinite(t) or abs(t) >= 2.0 ** 96:
            return math.nan
        q = int(Fraction(abs(t)) * 2 ** (-LSB))      # floor of |t| 2^192: truncation
        total += -q if t < 0 else q
    digits = []
    for _ in range(XD - 1):
        digits.append(total % (1 << 32))             # floor semantics, as the device's >> 32
        total >>= 32
    v = float(total)                                 # the signed top digit
    for d in reversed(digits):
        v = v * 4294967296.0 + float(d)
    return math.ldexp(v, LSB)
