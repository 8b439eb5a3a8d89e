"""CPU emulation of the CRT int8 Gram (csrc/kernels/gram_crt.hip): the moduli are pairwise coprime with a
product past 2 * 2^21 * 2^98 (exact reconstruction of any 2^21-row Gram of 49-bit integer images), the
Garner table compiled into the kernel is the modular-inverse table, and the kernel's arithmetic -- the
symmetric residues of the slicer (floor of n / p by a double product, one correction), the per-chunk
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
    assert len(mods) == len(inv) == 19 and all(m <= 127 and m % 2 == 1 for m in mods)
    for i in range(len(mods)):
        for j in range(i):
            assert math.gcd(mods[i], mods[j]) == 1
            assert inv[i][j] == pow(mods[j] % mods[i], -1, mods[i]), (i, j)
    M = reduce(lambda a, b: a * b, mods)
    assert max_rows * (2 ** kb) ** 2 < M // 2  # |G| < M / 2: the balanced reconstruction is exact


def _residue(nv: float, p: int) -> int:
    """crt_slice: floor(n / p) via a double product, an exact fma remainder, one correction, symmetric."""
    mp, ip = float(p), 1.0 / p
    qq = math.floor(nv * ip)
    r = nv - qq * mp  # exact in the kernel (fma); exact here too: |qq mp| < 2^51 integers
    if r < 0:
        r += mp
    if r >= mp:
        r -= mp
    if r > 0.5 * (mp - 1):
        r -= mp
    return int(r)


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
