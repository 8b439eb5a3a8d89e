"""CPU emulation of the CRT int8 Gram (csrc/kernels/gram_crt.hip): the moduli are pairwise coprime with a
product past 2 * 2^21 * 2^98 (exact reconstruction of any 2^21-row Gram of 49-bit integer images), the
Garner table compiled into the kernel is the modular-inverse table, and the kernel's arithmetic -- the
slicer's int8 residues (13-bit digits, exact f32 sums, an f32 quotient estimate, the residue read
from the low byte of a float's bit pattern; |r| <= 120), the per-chunk
reduction mod p, balanced Garner digits and the Horner evaluation in doubles -- reproduces the exact
integer Gram (Python integers) of random data including negative and boundary values."""
import math
import os
import re
from functools import reduce

import numpy as np

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "kernels", "gram_crt.hip")


def _tables():
    s = open(SRC).read()
    mods = [int(v) for v in re.search(r"constexpr int kMod\[NMOD\] = \{([^}]*)\}", s).group(1).split(",")]
    body = re.search(r"constexpr int kInv\[NMOD\]\[NMOD\] = \{(.*?)\};", s, re.S).group(1)
    rows = [[int(v) for v in r.split(",")] for r in re.findall(r"\{([^{}]*)\}", body)]
    kb = int(re.search(r"constexpr int KB = (\d+);", s).group(1))
    max_rows = 1 << int(re.search(r"MAX_ROWS = 1L << (\d+);", s).group(1))
    return mods, rows, kb, max_rows


def test_moduli_and_inverse_table():
    mods, inv, kb, max_rows = _tables()
    assert len(mods) == len(inv) == 16 and all(m <= 234 for m in mods)  # |r| <= 0.511 p fits int8
    for i in range(len(mods)):
        for j in range(i):
            assert math.gcd(mods[i], mods[j]) == 1
            assert inv[i][j] == pow(mods[j] % mods[i], -1, mods[i]), (i, j)
    M = reduce(lambda a, b: a * b, mods)
    assert max_rows * (2 ** kb) ** 2 < M // 2  # |G| < M / 2: the balanced reconstruction is exact


def _f32(x) -> np.float32:
    """Round an exact rational to the nearest f32 (an fma's single rounding)."""
    return np.float32(float(x))


MAGIC = 12582912  # 1.5 2^23


def _residue(nv: float, p: int) -> int:
    """crt_slice: N = d3 2^39 + d2 2^26 + d1 2^13 + d0 (13-bit digits, d3 signed), S' = MAGIC + d0 +
    d1 (2^13 mod p) + d2 (2^26 mod p) + d3 (2^39 mod p) in f32 (exact integers < 2^24), q = rint(fma(S',
    f32(1/p), f32(-MAGIC/p))), t = fma(-q, p, S') = MAGIC + r; r = the low byte of t's bits as int8."""
    from fractions import Fraction
    n = int(nv)
    d3 = math.floor(nv * 2.0 ** -39)
    r3 = n - d3 * 2 ** 39
    d2 = r3 >> 26
    r2 = r3 - (d2 << 26)
    d1, d0 = r2 >> 13, r2 & 8191
    assert -1024 <= d3 < 1024 and 0 <= d2 < 8192 and 0 <= d1 < 8192
    S = MAGIC + d0 + d1 * pow(2, 13, p) + d2 * pow(2, 26, p) + d3 * pow(2, 39, p)
    assert 2 ** 23 <= S < 2 ** 24  # exact in f32, exponent fixed
    ip, nm = np.float32(1.0) / np.float32(p), _f32(Fraction(-MAGIC, p))
    q = int(np.rint(_f32(Fraction(S) * Fraction(float(ip)) + Fraction(float(nm)))))
    t = S - q * p  # the fma is exact: an integer in [2^23, 2^24)
    assert 2 ** 23 <= t < 2 ** 24
    bits = int(np.array([t], dtype=np.float32).view(np.uint32)[0])
    r = bits & 0xFF
    r = r - 256 if r >= 128 else r
    assert r == t - MAGIC and (r - n) % p == 0 and abs(r) <= 120, (nv, p, r)
    return r


def _garner(res, mods, inv) -> float:
    v = []
    for i, mi in enumerate(mods):
        u = res[i]
        for j in range(i):
            u = int(math.fmod((u - v[j]) * inv[i][j], mi))  # C++ % (truncating)
        hm = mi >> 1
        if u > hm:
            u -= mi
        if u < -hm:
            u += mi
        v.append(u)
    val = float(v[-1])
    for i in range(len(mods) - 2, -1, -1):
        val = val * mods[i] + v[i]  # fma in the kernel; a double rounding here is within the tolerance
    return val, v


def test_emulated_gram_is_exact():
    mods, inv, kb, _ = _tables()
    rng = np.random.default_rng(0)
    m, d = 300, 5
    N = rng.integers(-(2 ** kb) + 1, 2 ** kb, size=(m, d), dtype=np.int64)
    N[0, :] = 2 ** kb - 1          # extremes
    N[1, :] = -(2 ** kb) + 1
    N[2, 0] = 0
    chunk = 128                    # the kernel reduces mod p after every chunk
    for a in range(d):
        for b in range(a + 1):
            exact = sum(int(N[i, a]) * int(N[i, b]) for i in range(m))
            res = []
            for p in mods:
                acc = 0
                for c0 in range(0, m, chunk):
                    s = sum(_residue(float(N[i, a]), p) * _residue(float(N[i, b]), p) for i in range(c0, min(m, c0 + chunk)))
                    acc = int(math.fmod(acc + s, p))
                    hm = p >> 1
                    if acc > hm:
                        acc -= p
                    if acc < -hm:
                        acc += p
                res.append(acc)
            val, digits = _garner(res, mods, inv)
            # the balanced mixed-radix digits are exact
            P, tot = 1, 0
            for i, p in enumerate(mods):
                tot += digits[i] * P
                P *= p
            assert tot == exact, (a, b)
            assert abs(val - exact) <= 4e-16 * abs(exact) + 1.0, (a, b, val, exact)


def test_slicer_residue_bound_dense():
    """|r| <= 120 and r == N mod p over random and boundary 49-bit integers, every modulus."""
    mods, _, kb, _ = _tables()
    rng = np.random.default_rng(1)
    vals = list(rng.integers(-(2 ** kb) + 1, 2 ** kb, size=4000, dtype=np.int64))
    vals += [0, 1, -1, 2 ** kb - 1, -(2 ** kb) + 1, 2 ** 24, -(2 ** 24), 2 ** 34 - 1, -(2 ** 34) + 1]
    vals += list(rng.integers(-2 ** 20, 2 ** 20, size=2000, dtype=np.int64))
    for p in mods:
        for v in vals:
            _residue(float(v), p)
