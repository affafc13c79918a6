"""ctypes binding of oracle/_build/libgroth16_cpu.so (C++ CPU restatement) —
TEST INFRASTRUCTURE ONLY; see oracle/__init__.py and oracle/cpu/groth16_cpu.cpp."""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "libgroth16_cpu.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError("C++ oracle not built: make -C oracle")
        L = ctypes.CDLL(LIB)
        u8p = ctypes.c_char_p
        L.g16cpu_prove.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, u8p, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        L.g16cpu_msm_g1.argtypes = [u8p, u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        L.g16cpu_msm_g2.argtypes = [u8p, u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        L.g16cpu_ntt.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _lib = L
    return _lib


def _ints(raw, k):
    return [int.from_bytes(raw[32 * i:32 * i + 32], "little") for i in range(k)]


def prove(zkey, wtns, r: int, s: int, threads: int = 8, zkey_ptr=None, zkey_len=None):
    """Returns ((ax, ay), ((bx0, bx1), (by0, by1)), (cx, cy)), stage ms [abc, ntt, g1, g2, total]."""
    out = ctypes.create_string_buffer(256)
    ms = (ctypes.c_double * 5)()
    if zkey_ptr is not None:
        zp, zl = ctypes.cast(zkey_ptr, ctypes.c_char_p), zkey_len
    else:
        zp, zl = zkey, len(zkey)
    lib().g16cpu_prove(zp, zl, wtns, len(wtns), int(r).to_bytes(32, "little"), int(s).to_bytes(32, "little"),
                       threads, out, ms)
    v = _ints(out.raw, 8)
    return ((v[0], v[1]), ((v[2], v[3]), (v[4], v[5])), (v[6], v[7])), list(ms)


def msm_g1(points: bytes, scalars: bytes, threads: int = 8):
    out = ctypes.create_string_buffer(64)
    lib().g16cpu_msm_g1(points, scalars, len(scalars) // 32, threads, out)
    v = _ints(out.raw, 2)
    return None if v == [0, 0] else tuple(v)


def msm_g2(points: bytes, scalars: bytes, threads: int = 8):
    out = ctypes.create_string_buffer(128)
    lib().g16cpu_msm_g2(points, scalars, len(scalars) // 32, threads, out)
    v = _ints(out.raw, 4)
    return None if v == [0, 0, 0, 0] else ((v[0], v[1]), (v[2], v[3]))


def ntt(values: bytes, mode: int, threads: int = 8) -> bytes:
    """Fr NTT of len(values) // 32 standard-form LE values (a power of two): mode 0 Fr.fft, 1 Fr.ifft,
    2 the coset extension ifft -> batchApplyKey(1, Fr.w[k+1]) -> fft (groth16_cpu.cpp g16cpu_ntt).
    Returns the outputs in the same layout."""
    n = len(values) // 32
    out = ctypes.create_string_buffer(len(values))
    if lib().g16cpu_ntt(values, n, mode, threads, out) != 0:
        raise ValueError("g16cpu_ntt: n must be a power of two <= 2^27 and mode 0..2")
    return out.raw
