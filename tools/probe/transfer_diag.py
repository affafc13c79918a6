#!/usr/bin/env python3
"""Diagnosis of an intermittent mismatch (tests/test_gpu_witness_transfer.py, all-large witness):
which of the five MSM sums is wrong.  (Found: the encoder's stray word past a full chunk landed in
the next chunk's metadata when that chunk had been encoded first -- wtns_pack.hpp WT_SLACK.)  For a few device-memory
states (fresh; device memory filled with a byte pattern through torch and released before the
prover is built), a one-part partial prover (zkp_prove_partial: the five MSM sums, no blinding)
is compared sum by sum with oracle/cpu's MSMs over the zkey's own sections; H is checked against
the MSM of the GPU quotient (and the quotient against a second prover's).
usage: transfer_diag.py -> one JSON line per state"""
import json
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))
import zkp_amd  # noqa: E402
from zkp_amd import synth  # noqa: E402
from oracle import cpu_oracle  # noqa: E402

NV = 3 * 65536 + 37


def sections(buf):
    n = struct.unpack_from("<I", buf, 8)[0]
    o, out = 12, {}
    for _ in range(n):
        sid, ln = struct.unpack_from("<IQ", buf, o)
        out[sid] = buf[o + 12:o + 12 + ln]
        o += 12 + ln
    return out


def g1(b):
    v = [int.from_bytes(b[32 * i:32 * i + 32], "little") for i in range(2)]
    return None if v == [0, 0] else tuple(v)


def g2(b):
    v = [int.from_bytes(b[32 * i:32 * i + 32], "little") for i in range(4)]
    return None if v == [0, 0, 0, 0] else ((v[0], v[1]), (v[2], v[3]))


def poison(byte):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    p = ctypes.c_void_p()
    n = ctypes.c_size_t(48 << 30)
    assert hip.hipMalloc(ctypes.byref(p), n) == 0
    assert hip.hipMemset(p, ctypes.c_int(byte), n) == 0
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipFree(p) == 0


def main():
    circ = synth.Circuit(NV, NV + 211, 26, 0x5A4B5032)
    zk = circ.zkey(0x5A4B5033).bytes()
    sec = sections(zk)
    w = circ.witness(91)
    off = len(w) - 32 * NV
    v = np.frombuffer(w, dtype=np.uint32, count=8 * NV, offset=off).reshape(NV, 8).copy()
    rng = np.random.default_rng(5)
    v[:] = rng.integers(0, 1 << 32, size=v.shape, dtype=np.uint64).astype(np.uint32)
    v[:, 7] &= 0x1FFFFFFF
    v[0] = 0
    v[0, 0] = 1
    w = w[:off] + v.tobytes()
    scal = v.tobytes()
    npub = 26
    want = {"a": cpu_oracle.msm_g1(sec[5], scal), "b1": cpu_oracle.msm_g1(sec[6], scal),
            "c": cpu_oracle.msm_g1(sec[8], scal[32 * (npub + 1):]), "b2": cpu_oracle.msm_g2(sec[7], scal)}
    full = zkp_amd.Prover(zk, devices=[0])
    q = full.quotient(w)
    full.close()
    qb = b"".join(x.to_bytes(32, "little") for x in q)
    want["h"] = cpu_oracle.msm_g1(sec[9], qb)
    for state in ("fresh", "poison_a5", "fresh_again", "poison_ff", "poison_00"):
        if state.startswith("poison"):
            poison(int(state[-2:], 16))
        p = zkp_amd.Prover(zk, devices=[0], part=0, nparts=1)
        res = {"state": state}
        for rep in range(2):
            pr = p.prove_partial(w)
            got = {"a": g1(pr[0:64]), "b1": g1(pr[64:128]), "c": g1(pr[128:192]), "h": g1(pr[192:256]),
                   "b2": g2(pr[256:384])}
            res["rep%d" % rep] = {k: got[k] == want[k] for k in want}
        try:
            q2 = p.quotient(w)
        except Exception:  # a partial prover may not offer the full quotient
            q2 = None
        p.close()
        res["quotient_equal"] = (q2 == q) if q2 is not None else None
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
