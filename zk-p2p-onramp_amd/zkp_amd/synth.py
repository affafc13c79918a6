"""Binding of libzkp_synth.so — TOOLING (synthetic Venmo-shaped circuits, witnesses
and insecure known-tau zkeys in snarkjs formats) for benchmarks and large tests.
Not the proving path.  See include/zkp_synth.h."""
from __future__ import annotations

import ctypes
import os

from . import PKG_ROOT, LibraryNotBuilt

LIB_PATH = os.path.join(PKG_ROOT, "lib", "libzkp_synth.so")
_lib = None

# Venmo circuit shape (README.md:79,83; nPublic from vkey.ts:4)
VENMO = dict(n_vars=6_400_562, n_constraints=6_618_823, n_public=26)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LibraryNotBuilt("libzkp_synth.so not found at %s" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.zkp_synth_circuit_new.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_uint64, ctypes.c_uint32,
                                                                     ctypes.POINTER(P)]
        L.zkp_synth_circuit_new_mix.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_uint64, ctypes.c_uint32,
                                                                         ctypes.c_uint32, ctypes.POINTER(P)]
        L.zkp_synth_circuit_free.argtypes = [P]
        L.zkp_synth_circuit_free.restype = None
        L.zkp_synth_domain_size.argtypes = [P]
        L.zkp_synth_domain_size.restype = ctypes.c_uint32
        L.zkp_synth_witness.argtypes = [P, ctypes.c_uint64, u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.zkp_synth_zkey.argtypes = [P, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(u8p),
                                     ctypes.POINTER(ctypes.c_size_t)]
        L.zkp_synth_zkey_ex.argtypes = [P, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]
        L.zkp_synth_r1cs.argtypes = [P, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]
        L.zkp_synth_ptau.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(u8p),
                                     ctypes.POINTER(ctypes.c_size_t)]
        L.zkp_synth_free.argtypes = [u8p]
        L.zkp_synth_free.restype = None
        L.zkp_synth_points_g1.argtypes = [ctypes.c_int, u8p, ctypes.c_size_t, u8p]
        L.zkp_synth_points_g2.argtypes = [ctypes.c_int, u8p, ctypes.c_size_t, u8p]
        L.zkp_synth_scalars.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, u8p]
        L.zkp_synth_scalars.restype = None
        L.zkp_synth_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _chk(rc):
    if rc != 0:
        raise RuntimeError("zkp_synth: " + lib().zkp_synth_last_error().decode())


class Circuit:
    def __init__(self, n_vars, n_constraints, n_public, seed, in_permille=50, bool_pct=70):
        """bool_pct: percent of bit-valued (AND/XOR) defining steps -- the witness-mix knob
        (70 = the default assumption; 0 = every defined signal uniform)."""
        h = ctypes.c_void_p()
        _chk(lib().zkp_synth_circuit_new_mix(n_vars, n_constraints, n_public, seed, in_permille, bool_pct,
                                             ctypes.byref(h)))
        self.bool_pct = bool_pct
        self._h = h
        self.n_vars, self.n_constraints, self.n_public = n_vars, n_constraints, n_public
        self.domain_size = lib().zkp_synth_domain_size(h)

    @classmethod
    def venmo(cls, seed=0x5A4B5032, bool_pct=70):
        return cls(VENMO["n_vars"], VENMO["n_constraints"], VENMO["n_public"], seed, bool_pct=bool_pct)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().zkp_synth_circuit_free(self._h)
            self._h = None

    def witness(self, wseed) -> bytes:
        n = ctypes.c_size_t()
        _chk(lib().zkp_synth_witness(self._h, wseed, None, 0, ctypes.byref(n)))
        buf = (ctypes.c_uint8 * n.value)()
        _chk(lib().zkp_synth_witness(self._h, wseed, ctypes.cast(buf, ctypes.POINTER(ctypes.c_uint8)), n.value,
                                     ctypes.byref(n)))
        return bytes(buf)

    def zkey(self, setup_seed, device=0, threads=0, unit_gamma_delta=False) -> "ZkeyBuffer":
        """Known-tau zkey; unit_gamma_delta: gamma = delta = 1, the key `zkey new` writes from
        ptau(power, setup_seed) (sections 2..9 equal zkp_zkey_new's)."""
        p = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        _chk(lib().zkp_synth_zkey_ex(self._h, setup_seed, 1 if unit_gamma_delta else 0, device, threads,
                                     ctypes.byref(p), ctypes.byref(n)))
        return ZkeyBuffer(p, n.value)

    def r1cs(self) -> "ZkeyBuffer":
        """The circuit as circom .r1cs bytes (library-owned buffer)."""
        p = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        _chk(lib().zkp_synth_r1cs(self._h, ctypes.byref(p), ctypes.byref(n)))
        return ZkeyBuffer(p, n.value)


def ptau(power, setup_seed, device=0, threads=0) -> "ZkeyBuffer":
    """A prepared known-tau .ptau of `power` (tau, alpha, beta of setup_seed as Circuit.zkey): every point
    section computed on the GPU (power 24 for the Venmo shape: ~17 GB).  INSECURE tooling."""
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _chk(lib().zkp_synth_ptau(power, setup_seed, device, threads, ctypes.byref(p), ctypes.byref(n)))
    return ZkeyBuffer(p, n.value)


class ZkeyBuffer:
    """Library-owned zkey bytes (can be GBs): pass .ptr/.len to zkp_prover_load_mem without copying."""

    def __init__(self, ptr, n):
        self.ptr, self.len = ptr, n

    def bytes(self) -> bytes:
        from . import _copy_out
        return _copy_out(self.ptr, self.len)

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().zkp_synth_free(self.ptr)
            self.ptr = None


def scalars(seed, stream, n) -> bytes:
    buf = (ctypes.c_uint8 * (32 * n))()
    lib().zkp_synth_scalars(seed, stream, n, ctypes.cast(buf, ctypes.POINTER(ctypes.c_uint8)))
    return bytes(buf)


def points(scalars_le: bytes, g2=False, device=0) -> bytes:
    n = len(scalars_le) // 32
    out = (ctypes.c_uint8 * (n * (128 if g2 else 64)))()
    src = (ctypes.c_uint8 * len(scalars_le)).from_buffer_copy(scalars_le)
    fn = lib().zkp_synth_points_g2 if g2 else lib().zkp_synth_points_g1
    _chk(fn(device, ctypes.cast(src, ctypes.POINTER(ctypes.c_uint8)), n, ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8))))
    return bytes(out)
