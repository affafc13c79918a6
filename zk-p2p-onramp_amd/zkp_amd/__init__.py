"""Python host binding of libzkp_amd.so — the MI355X-native Groth16 prover.

Mirrors the snarkjs interface this path replaces (snarkjs@0.4.22, reference
``package-lock.json:3884-3896``):

* ``groth16.prove(zkeyFileName, witnessFileName, logger=None)`` →
  ``{"proof": {...}, "publicSignals": [...]}`` — reference call sites
  ``app/src/helpers/zkp.ts:94`` (via fullProve) and
  ``dizkus-scripts/5_gen_proof.sh:8`` (CLI).  Inputs are a path or a fastfile
  memory descriptor ``{"type": "mem", "data": bytes}``.
* errors raise ``Error`` subclasses with snarkjs' messages ("zkey file is not
  groth16", "Invalid witness length...", ...).

The HIP library is REQUIRED: there is no CPU fallback.  Loading fails loudly
(``LibraryNotBuilt``) when ``lib/libzkp_amd.so`` is missing.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("ZKP_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libzkp_amd.so")  # override: A/B runs
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "zkp_amd.h")

ZKP_OK = 0
# BN254 scalar field order r (reference contracts/Verifier.sol:341)
R_MOD = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
STATUS_NAMES = {
    0: "ZKP_OK", 1: "ZKP_ERR_INVALID_ARG", 2: "ZKP_ERR_IO", 3: "ZKP_ERR_FORMAT", 4: "ZKP_ERR_PROTOCOL",
    5: "ZKP_ERR_CURVE", 6: "ZKP_ERR_WITNESS_LENGTH", 7: "ZKP_ERR_DEVICE", 8: "ZKP_ERR_OUT_OF_MEMORY",
    9: "ZKP_ERR_INTERNAL",
}


class LibraryNotBuilt(RuntimeError):
    pass


class ZkpError(Exception):
    def __init__(self, status: int, message: str):
        super().__init__("%s: %s" % (STATUS_NAMES.get(status, status), message))
        self.status = status
        self.message = message


class _Proof(ctypes.Structure):
    _fields_ = [
        ("pi_a", (ctypes.c_uint8 * 32) * 2),
        ("pi_b", ((ctypes.c_uint8 * 32) * 2) * 2),
        ("pi_c", (ctypes.c_uint8 * 32) * 2),
        ("n_public", ctypes.c_uint32),
        ("public_capacity", ctypes.c_uint32),
        ("public_signals", ctypes.POINTER(ctypes.c_uint8)),
    ]


_lib = None
_lib_lock = threading.Lock()


def load_library(path: str = LIB_PATH):
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise LibraryNotBuilt("libzkp_amd.so not found at %s — run __graft_entry__.build() "
                                  "(make -C zk-p2p-onramp_amd)" % path)
        lib = ctypes.CDLL(path)
        P = ctypes.c_void_p
        u8p = ctypes.POINTER(ctypes.c_uint8)
        sz = ctypes.c_size_t
        lib.zkp_prover_load_mem.argtypes = [u8p, sz, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(P)]
        lib.zkp_prover_load_file.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                             ctypes.POINTER(P)]
        lib.zkp_prover_info.argtypes = [P, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint32)]
        lib.zkp_prove.argtypes = [P, u8p, sz, u8p, u8p, ctypes.POINTER(_Proof)]
        lib.zkp_prove_batch.argtypes = [P, ctypes.POINTER(u8p), ctypes.POINTER(sz), ctypes.c_int,
                                        ctypes.POINTER(u8p), ctypes.POINTER(u8p), ctypes.POINTER(_Proof)]
        lib.zkp_prove_batch_status.argtypes = [P, ctypes.POINTER(u8p), ctypes.POINTER(sz), ctypes.c_int,
                                               ctypes.POINTER(u8p), ctypes.POINTER(u8p), ctypes.POINTER(_Proof),
                                               ctypes.POINTER(ctypes.c_int)]
        lib.zkp_prove_files.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        lib.zkp_proof_json.argtypes = [ctypes.POINTER(_Proof), ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        lib.zkp_public_json.argtypes = [ctypes.POINTER(_Proof), ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        lib.zkp_prover_timings.argtypes = [P, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
        lib.zkp_prover_free.argtypes = [P]
        lib.zkp_prover_free.restype = None
        lib.zkp_last_error.restype = ctypes.c_char_p
        lib.zkp_version.restype = ctypes.c_char_p
        lib.zkp_msm_g1.argtypes = [ctypes.c_int, u8p, u8p, sz, u8p, ctypes.POINTER(ctypes.c_int)]
        lib.zkp_msm_g2.argtypes = [ctypes.c_int, u8p, u8p, sz, u8p, ctypes.POINTER(ctypes.c_int)]
        lib.zkp_ntt_fr.argtypes = [ctypes.c_int, u8p, sz, ctypes.c_int]
        lib.zkp_quotient.argtypes = [P, u8p, sz, u8p]
        lib.zkp_witness_stage.argtypes = [P, ctypes.c_int, ctypes.c_int, u8p, sz]
        lib.zkp_prove_staged.argtypes = [P, ctypes.c_int, ctypes.c_int, u8p, u8p, ctypes.POINTER(_Proof)]
        lib.zkp_prover_instrument.argtypes = [P, ctypes.c_int]
        lib.zkp_prover_kernel_stats.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        lib.zkp_prover_launch_stats.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_int)]
        lib.zkp_bench_msm.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p, sz, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double), u8p, ctypes.POINTER(ctypes.c_int)]
        if hasattr(lib, "zkp_bench_msm_ex"):
            lib.zkp_bench_msm_ex.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p, sz, ctypes.c_int, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_double), ctypes.c_int, u8p,
                                             ctypes.POINTER(ctypes.c_int)]
        lib.zkp_bench_ntt.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double)]
        lib.zkp_bench_ntt_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_double)]
        lib.zkp_bench_plan.argtypes = [ctypes.c_int, u8p, sz, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        lib.zkp_msm.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p, sz, ctypes.c_int, ctypes.c_int, u8p,
                                ctypes.POINTER(ctypes.c_int)]
        lib.zkp_prover_msm_config.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        lib.zkp_proof_calldata.argtypes = [ctypes.POINTER(_Proof), ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        lib.zkp_prover_load_chunks.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(P)]
        lib.zkp_zkey_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(u8p), ctypes.POINTER(sz)]
        lib.zkp_zkey_read_chunks.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.POINTER(u8p),
                                             ctypes.POINTER(sz)]
        lib.zkp_zkey_contribute.argtypes = [ctypes.c_int, u8p, sz, u8p, ctypes.POINTER(u8p), ctypes.POINTER(sz)]
        lib.zkp_zkey_new.argtypes = [ctypes.c_int, u8p, sz, u8p, sz, ctypes.POINTER(u8p), ctypes.POINTER(sz)]
        lib.zkp_beacon_secret.argtypes = [u8p, sz, ctypes.c_uint32, u8p]
        lib.zkp_zkey_beacon.argtypes = [ctypes.c_int, u8p, sz, u8p, sz, ctypes.c_uint32, ctypes.POINTER(u8p),
                                        ctypes.POINTER(sz)]
        lib.zkp_buffer_free.argtypes = [u8p]
        lib.zkp_buffer_free.restype = None
        lib.zkp_prover_load_part.argtypes = [u8p, sz, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
        lib.zkp_prove_partial.argtypes = [P, u8p, sz, ctypes.c_char_p]
        lib.zkp_prove_partial_staged.argtypes = [P, ctypes.c_int, ctypes.c_char_p]
        lib.zkp_proof_combine.argtypes = [u8p, sz, ctypes.c_char_p, ctypes.c_int, u8p, sz, u8p, u8p,
                                          ctypes.POINTER(_Proof)]
        lib.zkp_quotient_part_staged.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
        lib.zkp_prove_partial_ext_staged.argtypes = [P, ctypes.c_int, ctypes.POINTER(P), ctypes.c_char_p]
        lib.zkp_zkey_beacon_named.argtypes = [ctypes.c_int, u8p, sz, u8p, sz, ctypes.c_uint32, ctypes.c_char_p,
                                              ctypes.POINTER(u8p), ctypes.POINTER(sz)]
        lib.zkp_zkey_contribute_entropy.argtypes = [ctypes.c_int, u8p, sz, u8p, ctypes.c_char_p, ctypes.c_char_p,
                                                    ctypes.POINTER(u8p), ctypes.POINTER(sz)]
        lib.zkp_blake2b512.argtypes = [u8p, sz, u8p]
        lib.zkp_prover_set_verify.argtypes = [P, ctypes.c_int]
        if hasattr(lib, "zkp_prover_get_verify"):  # round-5 entry points (an older library loads for A/B runs)
            lib.zkp_prover_get_verify.argtypes = [P, ctypes.POINTER(ctypes.c_int)]
        lib.zkp_proof_verify.argtypes = [u8p, sz, ctypes.POINTER(_Proof), ctypes.POINTER(ctypes.c_int)]
        lib.zkp_pairing.argtypes = [u8p, u8p, u8p]
        for name in ("zkp_zkey_beacon_named", "zkp_zkey_contribute_entropy", "zkp_blake2b512", "zkp_prover_set_verify", "zkp_prover_get_verify", "zkp_proof_verify", "zkp_pairing", "zkp_prover_load_mem", "zkp_prover_load_file", "zkp_prover_info", "zkp_prove",
                     "zkp_prove_batch", "zkp_prove_batch_status", "zkp_prove_files", "zkp_proof_json", "zkp_public_json",
                     "zkp_prover_timings", "zkp_msm_g1", "zkp_msm_g2", "zkp_ntt_fr", "zkp_quotient",
                     "zkp_witness_stage", "zkp_prove_staged", "zkp_prover_instrument", "zkp_prover_kernel_stats",
                     "zkp_prover_launch_stats",
                     "zkp_bench_msm", "zkp_bench_msm_ex", "zkp_bench_ntt", "zkp_bench_ntt_batch", "zkp_bench_plan", "zkp_msm", "zkp_prover_msm_config",
                     "zkp_prover_load_part", "zkp_prove_partial", "zkp_proof_calldata",
                     "zkp_prover_load_chunks", "zkp_zkey_read", "zkp_zkey_read_chunks", "zkp_zkey_contribute", "zkp_zkey_new",
                     "zkp_beacon_secret", "zkp_zkey_beacon", "zkp_prove_partial_staged", "zkp_proof_combine",
                     "zkp_quotient_part_staged", "zkp_prove_partial_ext_staged"):
            if hasattr(lib, name):
                getattr(lib, name).restype = ctypes.c_int
        _lib = lib
        return lib


def _check(st: int):
    if st != ZKP_OK:
        raise ZkpError(st, load_library().zkp_last_error().decode())


def _buf(data):
    """(ctypes uint8 pointer, keepalive) for a bytes-like object, without copying bytes /
    bytearray (witnesses are hundreds of MB; the C side only reads)."""
    if isinstance(data, bytes):
        return ctypes.cast(ctypes.c_char_p(data), ctypes.POINTER(ctypes.c_uint8)), data
    if isinstance(data, bytearray) and len(data):
        arr = (ctypes.c_uint8 * len(data)).from_buffer(data)
        return ctypes.cast(arr, ctypes.POINTER(ctypes.c_uint8)), arr
    data = bytes(data)
    return ctypes.cast(ctypes.c_char_p(data), ctypes.POINTER(ctypes.c_uint8)), data


def _copy_out(ptr, n: int) -> bytes:
    """bytes of a library buffer (ctypes.string_at takes a C int size: > 2 GiB needs a view)."""
    if n < (1 << 31) - 1:
        return ctypes.string_at(ptr, n)
    addr = ctypes.cast(ptr, ctypes.c_void_p).value
    return bytes(memoryview((ctypes.c_uint8 * n).from_address(addr)))


def _le(b) -> int:
    return int.from_bytes(bytes(b), "little")


def version() -> str:
    return load_library().zkp_version().decode()


class Prover:
    """A zkey resident in HBM of one or more devices (loaded once, reused per proof)."""

    def __init__(self, zkey, devices=None, part=None, nparts=None):
        """part / nparts: hold only point slice `part` of `nparts` on devices[0] (the
        point-range split of one proof over several GPUs) -> prove_partial only."""
        lib = load_library()
        h = ctypes.c_void_p()
        devs = list(devices or [])
        darr = (ctypes.c_int * max(1, len(devs)))(*devs) if devs else None
        dptr = ctypes.cast(darr, ctypes.POINTER(ctypes.c_int)) if darr is not None else None
        self.part, self.nparts = (part or 0), (nparts or 1)
        if nparts is not None:
            if hasattr(zkey, "ptr") and hasattr(zkey, "len"):
                _check(lib.zkp_prover_load_part(ctypes.cast(zkey.ptr, ctypes.POINTER(ctypes.c_uint8)), zkey.len,
                                                devs[0] if devs else 0, self.part, self.nparts, ctypes.byref(h)))
            else:
                if not isinstance(zkey, (bytes, bytearray, memoryview)):
                    zkey = open(zkey, "rb").read()
                p, keep = _buf(bytes(zkey))
                _check(lib.zkp_prover_load_part(p, len(zkey), devs[0] if devs else 0, self.part, self.nparts,
                                                ctypes.byref(h)))
                del keep
        elif hasattr(zkey, "ptr") and hasattr(zkey, "len"):  # library-owned buffer (e.g. synth.ZkeyBuffer)
            _check(lib.zkp_prover_load_mem(ctypes.cast(zkey.ptr, ctypes.POINTER(ctypes.c_uint8)), zkey.len, dptr,
                                           len(devs), ctypes.byref(h)))
        elif isinstance(zkey, (bytes, bytearray, memoryview)):
            p, keep = _buf(bytes(zkey))
            _check(lib.zkp_prover_load_mem(p, len(zkey), dptr, len(devs), ctypes.byref(h)))
            del keep
        else:
            _check(lib.zkp_prover_load_file(os.fsencode(zkey), dptr, len(devs), ctypes.byref(h)))
        self._h = h
        nv, npub, dom = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib.zkp_prover_info(h, ctypes.byref(nv), ctypes.byref(npub), ctypes.byref(dom)))
        self.n_vars, self.n_public, self.domain_size = nv.value, npub.value, dom.value

    def close(self):
        if getattr(self, "_h", None):
            load_library().zkp_prover_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _new_proof(self):
        pub = (ctypes.c_uint8 * (32 * max(1, self.n_public)))()
        pr = _Proof()
        pr.public_capacity = self.n_public
        pr.public_signals = ctypes.cast(pub, ctypes.POINTER(ctypes.c_uint8))
        return pr, pub

    @staticmethod
    def _scalar(x):
        if x is None:
            return None, None
        return _buf(int(x).to_bytes(32, "little"))

    def prove_raw(self, wtns: bytes, r=None, s=None):
        """Returns ((ax, ay), ((bx0, bx1), (by0, by1)), (cx, cy)), [public ints]."""
        lib = load_library()
        wp, wk = _buf(wtns)
        rp, rk = self._scalar(r)
        sp, sk = self._scalar(s)
        pr, pub = self._new_proof()
        _check(lib.zkp_prove(self._h, wp, len(wtns), rp, sp, ctypes.byref(pr)))
        return _unpack_proof(pr, pub)

    def prove_batch_raw(self, wtns_list, rs=None, ss=None):
        """All proofs of a batch (raises ZkpError if any proof failed)."""
        res, st = self._batch(wtns_list, rs, ss, raise_first=True)
        return res

    def prove_batch_status_raw(self, wtns_list, rs=None, ss=None):
        """(results, statuses): results[i] is None where statuses[i] != 0 (zkp_prove_batch_status:
        every proof attempted, device failures re-queued to the remaining devices)."""
        return self._batch(wtns_list, rs, ss, raise_first=False)

    def _batch(self, wtns_list, rs, ss, raise_first):
        lib = load_library()
        n = len(wtns_list)
        keep = []
        wps = (ctypes.POINTER(ctypes.c_uint8) * max(1, n))()
        lens = (ctypes.c_size_t * max(1, n))()
        for i, w in enumerate(wtns_list):
            p, k = _buf(w)
            keep.append(k)
            wps[i] = p
            lens[i] = len(w)

        def arr(vals):
            if vals is None:
                return None
            a = (ctypes.POINTER(ctypes.c_uint8) * max(1, n))()
            for i, v in enumerate(vals):
                p, k = _buf(int(v).to_bytes(32, "little"))
                keep.append(k)
                a[i] = p
            return a

        ra, sa = arr(rs), arr(ss)
        proofs = (_Proof * max(1, n))()
        pubs = []
        for i in range(n):
            pub = (ctypes.c_uint8 * (32 * max(1, self.n_public)))()
            pubs.append(pub)
            proofs[i].public_capacity = self.n_public
            proofs[i].public_signals = ctypes.cast(pub, ctypes.POINTER(ctypes.c_uint8))
        st = (ctypes.c_int * max(1, n))()
        rc = lib.zkp_prove_batch_status(self._h, wps, lens, n, ra, sa, proofs, st)
        if rc != ZKP_OK and raise_first:
            _check(rc)
        statuses = [st[i] for i in range(n)]
        return [_unpack_proof(proofs[i], pubs[i]) if statuses[i] == ZKP_OK else None for i in range(n)], statuses

    def prove(self, wtns: bytes, r=None, s=None):
        """snarkjs-shaped result {"proof": {...}, "publicSignals": [...]} (decimal strings)."""
        (a, b, c), pub = self.prove_raw(wtns, r, s)
        return {"proof": proof_object(a, b, c), "publicSignals": [str(x) for x in pub]}

    def quotient(self, wtns: bytes):
        lib = load_library()
        wp, wk = _buf(wtns)
        out = (ctypes.c_uint8 * (32 * self.domain_size))()
        _check(lib.zkp_quotient(self._h, wp, len(wtns), ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8))))
        raw = bytes(out)
        return [_le(raw[32 * i:32 * i + 32]) for i in range(self.domain_size)]

    def timings(self):
        lib = load_library()
        ms = (ctypes.c_float * 11)()
        _check(lib.zkp_prover_timings(self._h, ms, 11))
        keys = ["wtns_h2d", "build_abc", "ntt_quotient", "msm_g1_abc", "msm_g2", "host_assembly", "total_wall",
                "msm_g1_h", "verify", "wtns_pcie_mb", "witness_config"]
        return dict(zip(keys, list(ms)))

    VERIFY_OFF, VERIFY_ALL, VERIFY_BATCH = 0, 1, 2

    def set_verify(self, on=True):
        """Verify-before-return (zkp_prover_set_verify): a checked proof is verified by the host pairing
        against the zkey's verification key; a failing proof raises ZkpError (ZKP_ERR_INTERNAL), or has
        that status in a batch.  True / 1: every proof; False / 0: none; 2 (the default at load): the
        proofs of prove_batch* only."""
        mode = on if isinstance(on, int) and not isinstance(on, bool) else (1 if on else 0)
        _check(load_library().zkp_prover_set_verify(self._h, mode))

    def verify_mode(self) -> int:
        m = ctypes.c_int(-1)
        _check(load_library().zkp_prover_get_verify(self._h, ctypes.byref(m)))
        return m.value

    def stage(self, wtns: bytes, slot: int, dev_index: int = 0):
        wp, wk = _buf(wtns)
        _check(load_library().zkp_witness_stage(self._h, dev_index, slot, wp, len(wtns)))

    def prove_staged_raw(self, slot: int, r=None, s=None, dev_index: int = 0):
        rp, rk = self._scalar(r)
        sp, sk = self._scalar(s)
        pr, pub = self._new_proof()
        _check(load_library().zkp_prove_staged(self._h, dev_index, slot, rp, sp, ctypes.byref(pr)))
        return _unpack_proof(pr, pub)

    def instrument(self, on: bool = True):
        _check(load_library().zkp_prover_instrument(self._h, 1 if on else 0))

    def prove_partial(self, wtns: bytes) -> bytes:
        """This prover's slice of the five MSMs for one witness: a 392-byte zkp_partial."""
        wp, wk = _buf(wtns)
        out = ctypes.create_string_buffer(PARTIAL_BYTES)
        _check(load_library().zkp_prove_partial(self._h, wp, len(wtns), out))
        return out.raw

    def prove_partial_staged(self, slot: int) -> bytes:
        out = ctypes.create_string_buffer(PARTIAL_BYTES)
        _check(load_library().zkp_prove_partial_staged(self._h, slot, out))
        return out.raw

    def quotient_part_staged(self, slot: int, mask: int, dst_ptrs):
        """Distributed quotient, stage 1 (zkp_quotient_part_staged): coset extensions of the
        vectors in mask (bit 0 A, 1 B, 2 C) of the witness staged in `slot`, each copied to
        the device pointer dst_ptrs[v] (domain_size x 32 bytes; None for unselected)."""
        arr = (ctypes.c_void_p * 3)(*[p or None for p in dst_ptrs])
        _check(load_library().zkp_quotient_part_staged(self._h, slot, mask, arr))

    def prove_partial_ext_staged(self, slot: int, abc_ptrs) -> bytes:
        """Distributed quotient, stage 2 (zkp_prove_partial_ext_staged): this slice's
        partial sums with the H scalars joined from device pointers abc_ptrs[0..2] (A, B, C
        at this part's domain slice)."""
        arr = (ctypes.c_void_p * 3)(*abc_ptrs)
        out = ctypes.create_string_buffer(PARTIAL_BYTES)
        _check(load_library().zkp_prove_partial_ext_staged(self._h, slot, arr, out))
        return out.raw

    def msm_config(self):
        out = (ctypes.c_double * 10)()
        _check(load_library().zkp_prover_msm_config(self._h, out, 10))
        v = list(out)
        return {"witness": {"c": int(v[0]), "depth": int(v[1]), "groups": int(v[2])},
                "h": {"c": int(v[3]), "depth": int(v[4]), "groups": int(v[5])},
                "table_bytes_per_device": int(v[6]),
                "witness_second": ({"c": int(v[7]), "depth": int(v[8]), "groups": int(v[9])} if v[7] else None)}

    def kernel_stats(self):
        out = (ctypes.c_double * 8)()
        _check(load_library().zkp_prover_kernel_stats(self._h, out, 8))
        v = list(out)
        return {"g1": {"accumulate_ms": v[0], "launches": int(v[1]), "mixed_adds": int(v[2]), "tasks": int(v[3])},
                "g2": {"accumulate_ms": v[4], "launches": int(v[5]), "mixed_adds": int(v[6]), "tasks": int(v[7])}}

    LAUNCH_KINDS = ("A", "B1", "C", "H", "B2")

    def launch_stats(self):
        """Every instrumented accumulate launch: [{"msm": "A"|"B1"|"C"|"H"|"B2", "adds": n, "ms": t,
        "blocks": workgroups}]."""
        lib = load_library()
        n = ctypes.c_int(0)
        _check(lib.zkp_prover_launch_stats(self._h, None, 0, ctypes.byref(n)))
        cap = n.value
        out = (ctypes.c_double * (4 * max(1, cap)))()
        _check(lib.zkp_prover_launch_stats(self._h, out, cap, ctypes.byref(n)))
        v = list(out)
        # a proof finishing between the two calls grows the record count: read only what fits
        return [{"msm": self.LAUNCH_KINDS[int(v[4 * i])], "adds": int(v[4 * i + 1]), "ms": v[4 * i + 2],
                 "blocks": int(v[4 * i + 3])} for i in range(min(n.value, cap))]

    def prove_files(self, wtns_path, proof_path, public_path):
        _check(load_library().zkp_prove_files(self._h, os.fsencode(wtns_path), os.fsencode(proof_path),
                                              os.fsencode(public_path)))


def _unpack_proof(pr, pub):
    a = (_le(pr.pi_a[0]), _le(pr.pi_a[1]))
    b = ((_le(pr.pi_b[0][0]), _le(pr.pi_b[0][1])), (_le(pr.pi_b[1][0]), _le(pr.pi_b[1][1])))
    c = (_le(pr.pi_c[0]), _le(pr.pi_c[1]))
    raw = bytes(pub)
    signals = [_le(raw[32 * i:32 * i + 32]) for i in range(pr.n_public)]
    return (a, b, c), signals


def proof_object(a, b, c) -> dict:
    """snarkjs proof object (groth16_prove: pi_a, pi_b, pi_c, protocol, curve)."""
    return {
        "pi_a": [str(a[0]), str(a[1]), "1"],
        "pi_b": [[str(b[0][0]), str(b[0][1])], [str(b[1][0]), str(b[1][1])], ["1", "0"]],
        "pi_c": [str(c[0]), str(c[1]), "1"],
        "protocol": "groth16",
        "curve": "bn128",
    }


# ---------------------------------------------------------------- snarkjs-style module API

def _read_input(x) -> bytes:
    if isinstance(x, dict) and x.get("type") == "mem":
        return bytes(x["data"])
    if isinstance(x, (bytes, bytearray, memoryview)):
        return bytes(x)
    with open(x, "rb") as f:
        return f.read()


class _Groth16:
    """``groth16.prove`` with a per-process cache of loaded (HBM-resident) zkeys."""

    def __init__(self):
        self._cache = {}
        self._lock = threading.Lock()

    def _prover(self, zkey):
        key = zkey if isinstance(zkey, str) else id(zkey)
        with self._lock:
            p = self._cache.get(key)
            if p is None:
                p = Prover(zkey if isinstance(zkey, str) else _read_input(zkey))
                self._cache[key] = p
            return p

    def prove(self, zkeyFileName, witnessFileName, logger=None, r=None, s=None):
        p = self._prover(zkeyFileName)
        if logger is not None:
            logger.debug("zkp_amd: proving on device (nVars=%d, domain=%d)" % (p.n_vars, p.domain_size))
        return p.prove(_read_input(witnessFileName), r=r, s=s)


groth16 = _Groth16()

PARTIAL_BYTES = 392  # sizeof(zkp_partial)


def proof_combine_raw(zkey, partials, wtns: bytes, r=None, s=None):
    """Host-only: sum the partials (392-byte zkp_partial each, any order) of one split and
    assemble the proof -> same tuple as Prover.prove_raw."""
    lib = load_library()
    blob = b"".join(bytes(p) for p in partials)
    if len(blob) != PARTIAL_BYTES * len(partials):
        raise ValueError("each partial must be %d bytes" % PARTIAL_BYTES)
    if hasattr(zkey, "ptr") and hasattr(zkey, "len"):
        zp, zlen, zk = ctypes.cast(zkey.ptr, ctypes.POINTER(ctypes.c_uint8)), zkey.len, None
    else:
        if not isinstance(zkey, (bytes, bytearray, memoryview)):
            zkey = open(zkey, "rb").read()
        zp, zk = _buf(bytes(zkey))
        zlen = len(zkey)
    wp, wk = _buf(wtns)
    rp, rk = Prover._scalar(r)
    sp, sk = Prover._scalar(s)
    npub = 4096  # public-signal capacity (the Venmo circuit has 26)
    pub = (ctypes.c_uint8 * (32 * npub))()
    pr = _Proof()
    pr.public_capacity = npub
    pr.public_signals = ctypes.cast(pub, ctypes.POINTER(ctypes.c_uint8))
    _check(lib.zkp_proof_combine(zp, zlen, blob, len(partials), wp, len(wtns), rp, sp, ctypes.byref(pr)))
    if pr.n_public > npub:
        raise ZkpError(1, "more than %d public signals" % npub)
    return _unpack_proof(pr, pub)


def read_zkey(path_or_chunks) -> bytes:
    """Decompressed, merged zkey bytes (host only): a path (plain or gzip; else path.gz;
    else the chunks path{a..z}[.gz], the app's circuit.zkey{b..k}.gz) or a list of chunk paths."""
    lib = load_library()
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    if isinstance(path_or_chunks, (list, tuple)):
        arr = (ctypes.c_char_p * len(path_or_chunks))(*[os.fsencode(p) for p in path_or_chunks])
        _check(lib.zkp_zkey_read_chunks(arr, len(path_or_chunks), ctypes.byref(out), ctypes.byref(n)))
    else:
        _check(lib.zkp_zkey_read(os.fsencode(path_or_chunks), ctypes.byref(out), ctypes.byref(n)))
    try:
        return _copy_out(out, n.value)
    finally:
        lib.zkp_buffer_free(out)


def _in(buf):
    """(pointer, length, keepalive) of bytes or of a library-owned buffer (synth.ZkeyBuffer: .ptr / .len)."""
    if hasattr(buf, "ptr") and hasattr(buf, "len"):
        return ctypes.cast(buf.ptr, ctypes.POINTER(ctypes.c_uint8)), buf.len, buf
    p, k = _buf(bytes(buf) or b"\0")
    return p, len(buf), k


def zkey_contribute(zkey: bytes, k: int, device: int = 0) -> bytes:
    """Phase-2 contribution math on the GPU: delta -> k*delta (sections 2, 8, 9)."""
    lib = load_library()
    if hasattr(zkey, "ptr") and hasattr(zkey, "len"):  # library-owned buffer (synth.ZkeyBuffer)
        zp, zlen, zk = ctypes.cast(zkey.ptr, ctypes.POINTER(ctypes.c_uint8)), zkey.len, None
    else:
        zp, zk = _buf(zkey)
        zlen = len(zkey)
    kp, kk = _buf(int(k).to_bytes(32, "little"))
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib.zkp_zkey_contribute(device, zp, zlen, kp, ctypes.byref(out), ctypes.byref(n)))
    try:
        return _copy_out(out, n.value)
    finally:
        lib.zkp_buffer_free(out)


def beacon_secret(beacon: bytes, num_iterations_exp: int) -> int:
    """The contribution scalar of `snarkjs zkey beacon <beacon hex> <num_iterations_exp>`
    (host only: chained SHA-256, ChaCha20 stream, Fr.fromRng)."""
    lib = load_library()
    bp, bk = _buf(bytes(beacon) or b"\0")
    k = (ctypes.c_uint8 * 32)()
    _check(lib.zkp_beacon_secret(bp, len(beacon), num_iterations_exp, ctypes.cast(k, ctypes.POINTER(ctypes.c_uint8))))
    return int.from_bytes(bytes(k), "little")


def zkey_beacon(zkey: bytes, beacon: bytes, num_iterations_exp: int, device: int = 0, name=None) -> bytes:
    """`snarkjs zkey beacon <in> <out> <hex> <e> [-n=name]` (zkp_zkey_beacon_named): delta -> k*delta
    with k the beacon's secret on the GPU, the type-1 contribution record appended to section 10."""
    lib = load_library()
    zp, zlen, zk = _in(zkey)
    bp, bk = _buf(bytes(beacon) or b"\0")
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib.zkp_zkey_beacon_named(device, zp, zlen, bp, len(beacon), num_iterations_exp,
                                     name.encode() if name else None, ctypes.byref(out), ctypes.byref(n)))
    try:
        return _copy_out(out, n.value)
    finally:
        lib.zkp_buffer_free(out)


def zkey_contribute_entropy(zkey: bytes, entropy: str, rand64: bytes = None, name=None, device: int = 0) -> bytes:
    """`snarkjs zkey contribute <in> <out> -e=<entropy> [-n=name]` (zkp_zkey_contribute_entropy):
    rand64 = the 64 random bytes mixed with the entropy (None: /dev/urandom; tests pass fixed bytes)."""
    lib = load_library()
    zp, zlen, zk = _in(zkey)
    rp = None
    if rand64 is not None:
        if len(rand64) != 64:
            raise ValueError("rand64 must be 64 bytes")
        rp, rk = _buf(bytes(rand64))
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib.zkp_zkey_contribute_entropy(device, zp, zlen, rp, entropy.encode(), name.encode() if name else None,
                                           ctypes.byref(out), ctypes.byref(n)))
    try:
        return _copy_out(out, n.value)
    finally:
        lib.zkp_buffer_free(out)


def blake2b512(data: bytes) -> bytes:
    """Host-only Blake2b-512 of the C++ MPC code (zkp_blake2b512)."""
    dp, dk = _buf(bytes(data) or b"\0")
    out = (ctypes.c_uint8 * 64)()
    _check(load_library().zkp_blake2b512(dp, len(data), ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8))))
    return bytes(out)


def zkey_new(r1cs: bytes, ptau: bytes, device: int = 0) -> bytes:
    """`snarkjs zkey new`: the phase-2 starting key of a circom .r1cs from a prepared .ptau,
    point sections built on the GPU (zkp_zkey_new)."""
    lib = load_library()
    rp, rlen, rk = _in(r1cs)
    pp, plen, pk = _in(ptau)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib.zkp_zkey_new(device, rp, rlen, pp, plen, ctypes.byref(out), ctypes.byref(n)))
    try:
        return _copy_out(out, n.value)
    finally:
        lib.zkp_buffer_free(out)


def _proof_struct(proof, public_signals):
    (a, b, c) = proof
    pr = _Proof()
    for i in range(2):
        pr.pi_a[i][:] = int(a[i]).to_bytes(32, "little")
        pr.pi_c[i][:] = int(c[i]).to_bytes(32, "little")
        for j in range(2):
            pr.pi_b[i][j][:] = int(b[i][j]).to_bytes(32, "little")
    pub = b"".join(int(x).to_bytes(32, "little") for x in public_signals) or bytes(32)
    pbuf = (ctypes.c_uint8 * len(pub)).from_buffer_copy(pub)
    pr.n_public = pr.public_capacity = len(public_signals)
    pr.public_signals = ctypes.cast(pbuf, ctypes.POINTER(ctypes.c_uint8))
    return pr, pbuf


def proof_verify(zkey, proof, public_signals) -> bool:
    """Host-only `snarkjs groth16 verify` (zkp_proof_verify) of a proof tuple
    ((ax, ay), ((bx0, bx1), (by0, by1)), (cx, cy)) against a zkey's verification key."""
    if hasattr(zkey, "ptr") and hasattr(zkey, "len"):
        zp, zlen, zk = ctypes.cast(zkey.ptr, ctypes.POINTER(ctypes.c_uint8)), zkey.len, None
    else:
        zp, zk = _buf(bytes(zkey))
        zlen = len(zkey)
    pr, keep = _proof_struct(proof, public_signals)
    ok = ctypes.c_int()
    _check(load_library().zkp_proof_verify(zp, zlen, ctypes.byref(pr), ctypes.byref(ok)))
    return bool(ok.value)


def pairing(g1, g2):
    """Host-only BN254 pairing e(P, Q) in snarkjs' GT convention (zkp_pairing): P = (x, y),
    Q = ((x.c0, x.c1), (y.c0, y.c1)), None = infinity -> 6 x (c0, c1) ints in snarkjs' nesting."""
    gb = bytes(64) if g1 is None else b"".join(int(v).to_bytes(32, "little") for v in g1)
    qb = bytes(128) if g2 is None else b"".join(int(v).to_bytes(32, "little")
                                               for v in (g2[0][0], g2[0][1], g2[1][0], g2[1][1]))
    gp, gk = _buf(gb)
    qp, qk = _buf(qb)
    out = (ctypes.c_uint8 * 384)()
    _check(load_library().zkp_pairing(gp, qp, ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8))))
    raw = bytes(out)
    v = [_le(raw[32 * i:32 * i + 32]) for i in range(12)]
    return [[(v[6 * h + 2 * k], v[6 * h + 2 * k + 1]) for k in range(3)] for h in range(2)]


def solidity_calldata(proof, public_signals) -> str:
    """`snarkjs zkey export soliditycalldata` text via the C ABI (zkp_proof_calldata).
    proof: ((ax, ay), ((bx0, bx1), (by0, by1)), (cx, cy)) as from Prover.prove_raw."""
    (a, b, c) = proof
    pr = _Proof()
    for i in range(2):
        pr.pi_a[i][:] = int(a[i]).to_bytes(32, "little")
        pr.pi_c[i][:] = int(c[i]).to_bytes(32, "little")
        for j in range(2):
            pr.pi_b[i][j][:] = int(b[i][j]).to_bytes(32, "little")
    pub = b"".join(int(x).to_bytes(32, "little") for x in public_signals) or bytes(32)
    pbuf = (ctypes.c_uint8 * len(pub)).from_buffer_copy(pub)
    pr.n_public = pr.public_capacity = len(public_signals)
    pr.public_signals = ctypes.cast(pbuf, ctypes.POINTER(ctypes.c_uint8))
    need = ctypes.c_size_t()
    lib = load_library()
    _check(lib.zkp_proof_calldata(ctypes.byref(pr), None, 0, ctypes.byref(need)))
    out = ctypes.create_string_buffer(need.value)
    _check(lib.zkp_proof_calldata(ctypes.byref(pr), out, need.value, ctypes.byref(need)))
    return out.value.decode()


def partial_from_points(a, b1, c, h, b2, part: int, nparts: int) -> bytes:
    """Encode affine partial sums (oracle tuples, None = infinity) as a zkp_partial."""
    def g1(p):
        return bytes(64) if p is None else int(p[0]).to_bytes(32, "little") + int(p[1]).to_bytes(32, "little")

    def g2(p):
        if p is None:
            return bytes(128)
        return b"".join(int(v).to_bytes(32, "little") for v in (p[0][0], p[0][1], p[1][0], p[1][1]))
    return g1(a) + g1(b1) + g1(c) + g1(h) + g2(b2) + int(part).to_bytes(4, "little") + int(nparts).to_bytes(4, "little")


def _msm(points_lem, scalars_le, g2, device, window_bits, table_depth):
    lib = load_library()
    n = len(scalars_le) // 32
    pp, pk = _buf(points_lem)
    sp, sk = _buf(scalars_le)
    out = (ctypes.c_uint8 * 128)()
    inf = ctypes.c_int()
    o = ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8))
    if window_bits or table_depth:
        _check(lib.zkp_msm(device, 1 if g2 else 0, pp, sp, n, window_bits, table_depth, o, ctypes.byref(inf)))
    elif g2:
        _check(lib.zkp_msm_g2(device, pp, sp, n, o, ctypes.byref(inf)))
    else:
        _check(lib.zkp_msm_g1(device, pp, sp, n, o, ctypes.byref(inf)))
    if inf.value:
        return None
    raw = bytes(out)
    v = [_le(raw[32 * i:32 * i + 32]) for i in range(4)]
    return ((v[0], v[1]), (v[2], v[3])) if g2 else (v[0], v[1])


def msm_g1(points_lem: bytes, scalars_le: bytes, device: int = 0, window_bits: int = 0, table_depth: int = 0):
    """Kernel-level G1 MSM: zkey-layout points, 32-byte LE scalars -> affine (x, y) or None.
    window_bits / table_depth: Pippenger parameters (0 = automatic, as the prover)."""
    return _msm(points_lem, scalars_le, False, device, window_bits, table_depth)


def msm_g2(points_lem: bytes, scalars_le: bytes, device: int = 0, window_bits: int = 0, table_depth: int = 0):
    """Kernel-level G2 MSM -> ((x.c0, x.c1), (y.c0, y.c1)) or None."""
    return _msm(points_lem, scalars_le, True, device, window_bits, table_depth)


def ntt_fr(values, mode: int, device: int = 0):
    """mode 0 forward, 1 inverse, 2 coset-extend (snarkjs ifft -> applyKey -> fft)."""
    lib = load_library()
    raw = b"".join(int(v).to_bytes(32, "little") for v in values)
    arr = (ctypes.c_uint8 * len(raw)).from_buffer_copy(raw)
    _check(lib.zkp_ntt_fr(device, ctypes.cast(arr, ctypes.POINTER(ctypes.c_uint8)), len(values), mode))
    out = bytes(arr)
    return [_le(out[32 * i:32 * i + 32]) for i in range(len(values))]


def ntt_fr_bytes(raw, mode: int, device: int = 0) -> bytes:
    """As ntt_fr on len(raw) // 32 standard-form LE values (< r) given as bytes; returns bytes of the same
    layout (no per-element Python integers: the 2^20 / 2^23 parity tests)."""
    lib = load_library()
    arr = (ctypes.c_uint8 * len(raw)).from_buffer_copy(raw)
    _check(lib.zkp_ntt_fr(device, ctypes.cast(arr, ctypes.POINTER(ctypes.c_uint8)), len(raw) // 32, mode))
    return bytes(arr)


def bench_msm(points_lem: bytes, scalars_le: bytes, g2: bool = False, warmup: int = 2, iters: int = 10,
              device: int = 0):
    """Device-resident MSM timing (HIP events on the engine stream).  Returns (stats dict, result)."""
    lib = load_library()
    n = len(scalars_le) // 32
    pp, pk = _buf(points_lem)
    sp, sk = _buf(scalars_le)
    st = (ctypes.c_double * 8)()
    out = (ctypes.c_uint8 * 128)()
    inf = ctypes.c_int()
    ext = hasattr(lib, "zkp_bench_msm_ex")  # an older library (A/B runs) has the 6-stat form only
    if ext:
        _check(lib.zkp_bench_msm_ex(device, 1 if g2 else 0, pp, sp, n, warmup, iters, st, 8,
                                    ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(inf)))
    else:
        _check(lib.zkp_bench_msm(device, 1 if g2 else 0, pp, sp, n, warmup, iters, st,
                                 ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(inf)))
    raw = bytes(out)
    if inf.value:
        res = None
    elif g2:
        v = [_le(raw[32 * i:32 * i + 32]) for i in range(4)]
        res = ((v[0], v[1]), (v[2], v[3]))
    else:
        res = (_le(raw[:32]), _le(raw[32:64]))
    stats = {"ms_per_msm": st[0], "ms_accumulate": st[1], "mixed_adds": int(st[2]), "tasks": int(st[3]),
             "c": int(st[4]), "windows": int(st[5]), "table_build_ms": st[6] if ext else None,
             "table_depth": int(st[7]) if ext else None}
    return stats, res


def bench_plan(scalars_le: bytes, window_bits: int = 0, dense: bool = True, warmup: int = 2, iters: int = 10,
               device: int = 0) -> float:
    """ms per MSM plan build (digits + bucket grouping + task offsets), device-resident scalars."""
    ms = ctypes.c_double()
    sp, sk = _buf(scalars_le)
    _check(load_library().zkp_bench_plan(device, sp, len(scalars_le) // 32, window_bits, 1 if dense else 0, warmup,
                                         iters, ctypes.byref(ms)))
    return ms.value


def bench_ntt(log_n: int, warmup: int = 2, iters: int = 10, device: int = 0, count: int = 1) -> float:
    """ms per coset extension of `count` (1..3) vectors of 2^log_n elements, every pass one launch
    over all of them (count 3 is the prover's A, B, C)."""
    ms = ctypes.c_double()
    if count == 1:
        _check(load_library().zkp_bench_ntt(device, log_n, warmup, iters, ctypes.byref(ms)))
    else:
        _check(load_library().zkp_bench_ntt_batch(device, log_n, count, warmup, iters, ctypes.byref(ms)))
    return ms.value
