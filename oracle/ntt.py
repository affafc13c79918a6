"""Fr NTT in the ffjavascript convention — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates ``Fr.fft`` / ``Fr.ifft`` / ``Fr.batchApplyKey`` as snarkjs 0.4.22
``groth16_prove`` uses them (SURVEY.md §8a rows A5–A7; upstream pin
``package-lock.json:2060-2071``):

* roots: ``Fr.w[s] = nqr^t`` with nqr the smallest quadratic non-residue (5) and
  ``r - 1 = 2^s * t`` (s = 28); ``Fr.w[k] = Fr.w[k+1]^2``  (SURVEY App. B).
* ``fft(a)``  : natural order in/out, ``A_j = sum_i a_i w^(ij)``, w = Fr.w[log2 n].
* ``ifft(A)`` : natural order in/out, ``a_i = n^-1 sum_j A_j w^(-ij)``.
* coset key: ``g = Fr.w[log2 n + 1]`` (``Fr.shift`` only when log2 n == 28).
"""
from __future__ import annotations

from .bn254 import R, inv

TWO_ADICITY = 28


def _find_nqr() -> int:
    x = 2
    while pow(x, (R - 1) // 2, R) != R - 1:
        x += 1
    return x


NQR = _find_nqr()  # == 5
_T = (R - 1) >> TWO_ADICITY
ROOTS = [0] * (TWO_ADICITY + 1)
ROOTS[TWO_ADICITY] = pow(NQR, _T, R)
for _k in range(TWO_ADICITY - 1, -1, -1):
    ROOTS[_k] = ROOTS[_k + 1] * ROOTS[_k + 1] % R
FR_SHIFT = NQR * NQR % R


def log2_exact(n: int) -> int:
    k = n.bit_length() - 1
    if (1 << k) != n:
        raise ValueError("not a power of two: %d" % n)
    return k


def coset_gen(n: int) -> int:
    k = log2_exact(n)
    return FR_SHIFT if k == TWO_ADICITY else ROOTS[k + 1]


def _bitrev_permute(a):
    n = len(a)
    j = 0
    for i in range(1, n):
        bit = n >> 1
        while j & bit:
            j ^= bit
            bit >>= 1
        j |= bit
        if i < j:
            a[i], a[j] = a[j], a[i]


def _dft_inplace(a, w):
    """Iterative radix-2 DIT, natural in / natural out, A_j = sum a_i w^(ij)."""
    n = len(a)
    _bitrev_permute(a)
    m = 1
    while m < n:
        wm = pow(w, n // (2 * m), R)
        for k in range(0, n, 2 * m):
            t = 1
            for j in range(m):
                u = a[k + j]
                v = a[k + j + m] * t % R
                a[k + j] = (u + v) % R
                a[k + j + m] = (u - v) % R
                t = t * wm % R
        m *= 2


def fft(a):
    n = len(a)
    out = [x % R for x in a]
    if n > 1:
        _dft_inplace(out, ROOTS[log2_exact(n)])
    return out


def ifft(a):
    n = len(a)
    out = [x % R for x in a]
    if n > 1:
        _dft_inplace(out, inv(ROOTS[log2_exact(n)], R))
    ninv = inv(n, R)
    return [x * ninv % R for x in out]


def batch_apply_key(a, first: int, inc: int):
    """x_i <- x_i * first * inc^i (ffjavascript Fr.batchApplyKey)."""
    out = []
    cur = first % R
    for x in a:
        out.append(x * cur % R)
        cur = cur * inc % R
    return out


def naive_dft(a, w):
    n = len(a)
    return [sum(a[i] * pow(w, i * j, R) for i in range(n)) % R for j in range(n)]
