"""TEST INFRASTRUCTURE (oracle) -- the phase-2 MPC record of a snarkjs@0.4.22 zkey (section 10):
the circuit hash written by `zkey new`, the contribution entries appended by `zkey contribute` /
`zkey beacon`, and `zkey verify`, which accepts a key only if its transcript is consistent with
the initial key of the same circuit.

Reference call sites: dizkus-scripts/3_gen_chunk_zkey.sh:18 (`groth16 setup`), :27 (`zkey
contribute`), :36 (`zkey beacon ... 10 -n="Final Beacon phase2"`), and the gate
circuit/scripts/generate_keys_phase2_groth16.sh:26 (`zkey verify`).  The algorithms live in
snarkjs@0.4.22 (package-lock.json:3884-3896: zkey_new.js, zkey_contribute.js, zkey_beacon.js,
zkey_verify_frominit.js, zkey_utils.js read/writeMPCParams, keypair.js hashToG2, misc.js) and
ffjavascript 0.2.55 (ChaCha, F.fromRng, G.fromRng, toRprUncompressed) -- absent offline, restated
from their published source (recalled).  No zkey written by snarkjs is in the reference, so the
transcript BYTES are parity unpinned; the restatement is checked for internal consistency (every
key the GPU builds verifies here, tampered keys do not) and its primitives are pinned where a
fixture exists (Blake2b-512 and SHA-256 are hashlib; ChaCha20 against OpenSSL, beacon.py).

Recalled conventions:
* csHash = Blake2b-512 over, in order: alpha1, beta1, beta2, gamma2 (= G2), delta1 (= G1),
  delta2 (= G2) of the new key; then per point section a big-endian u32 count and the points:
  IC (nPublic + 1), H as (tau^(n+i) - tau^i) G1 from the ptau's tauG1 (count n - 1, hashed by
  chunks of min(n - 1, 2^14) points: the last chunk may read past n - 1), C (nVars - nPublic - 1),
  A, B1 (nVars each), B2 (nVars).  Points are "uncompressed": big-endian x || y, an Fq2 as
  c1 || c0; the point at infinity is zero bytes with the first byte 0x40.
* section 10 = csHash (64) || u32 count || per contribution: deltaAfter, g1_s, g1_sx (G1, LEM),
  g2_spx (G2, LEM), transcript (64), u32 type, u32 len || params (1: name, 2: numIterationsExp,
  3: beacon hash; each id, length byte(s), bytes).
* a contribution with secret k drawn from a ChaCha rng: k = Fr.fromRng, g1_s = G1.fromRng,
  g1_sx = k g1_s, transcript = Blake2b(csHash || pubkeys of the earlier contributions || g1_s U ||
  g1_sx U), g2_sp = G2.fromRng(ChaCha(first 8 big-endian words of the transcript)), g2_spx =
  k g2_sp; delta -> k delta, L and H -> k^-1 (setup.contribute_delta); deltaAfter = the new delta1.
  The rng: the beacon's (beacon.py) or, for `zkey contribute`, ChaCha(Blake2b(64 random bytes ||
  entropy text)).
* G.fromRng: x = F.fromRng (Montgomery reading), greatest = rng bit; redraw while x^3 + b is a
  non-residue; y = sqrt, negated unless (y > (p-1)/2) == greatest; G2 then times its cofactor 2p - r.
  An Fq2 value is "negative" by its c1, or by c0 when c1 = 0.
"""
from __future__ import annotations

import hashlib
import random
import struct

from . import bn254
from .beacon import ChaCha, MASK254, beacon_hash

P, R = bn254.P, bn254.R
RINV = pow(1 << 256, -1, P)
G2_COFACTOR = 2 * P - R
HALF_P = (P - 1) // 2
H_CHUNK = 1 << 14


def blake2b():
    return hashlib.blake2b(digest_size=64)


# ------------------------------------------------------------------ encodings

def g1_u(pt) -> bytes:
    if pt is None:
        return bytes([0x40]) + bytes(63)
    return pt[0].to_bytes(32, "big") + pt[1].to_bytes(32, "big")


def g2_u(pt) -> bytes:
    if pt is None:
        return bytes([0x40]) + bytes(127)
    (x0, x1), (y0, y1) = pt
    return b"".join(v.to_bytes(32, "big") for v in (x1, x0, y1, y0))


def u32be(n: int) -> bytes:
    return struct.pack(">I", n)


# ------------------------------------------------------------------ csHash (zkey new)

def cs_hash(z, tau: int) -> bytes:
    """csHash of the new key z (gamma = delta = 1) built from a ptau of toxic tau."""
    n = z.domain_size
    h = blake2b()
    for part in (g1_u(z.alpha1), g1_u(z.beta1), g2_u(z.beta2), g2_u(bn254.G2_GEN), g1_u(bn254.G1_GEN),
                 g2_u(bn254.G2_GEN)):
        h.update(part)
    h.update(u32be(len(z.ic)))
    for p in z.ic:
        h.update(g1_u(p))
    # H: (tau^(n+i) - tau^i) G1 = (tau^n - 1) tau^i G1, by chunks (recalled loop: every chunk has
    # min(n - 1, 2^14) points)
    h.update(u32be(n - 1))
    zt = (pow(tau, n, R) - 1) % R
    g1 = bn254.FixedBase(bn254.G1_GEN)
    i = 0
    while i < n - 1:
        m = min(n - 1, H_CHUNK)
        pts = bn254.batch_to_affine_g1([g1.mul_jac(zt * pow(tau, j, R) % R) for j in range(i, i + m)])
        for p in pts:
            h.update(g1_u(p))
        i += H_CHUNK
    for sec in (z.c, z.a, z.b1):
        h.update(u32be(len(sec)))
        for p in sec:
            h.update(g1_u(p))
    h.update(u32be(len(z.b2)))
    for p in z.b2:
        h.update(g2_u(p))
    return h.digest()


# ------------------------------------------------------------------ rng draws (ffjavascript)

def fq_from_rng(rng: ChaCha) -> int:
    while True:
        v = 0
        for i in range(4):
            v += rng.next_u64() << (64 * i)
        v &= MASK254
        if v < P:
            return v * RINV % P


def fr_from_rng(rng: ChaCha) -> int:
    from .beacon import fr_from_rng as f
    return f(rng)


def _neg_fq(y: int) -> bool:
    return y > HALF_P


def _neg_fq2(y) -> bool:
    return _neg_fq(y[1]) if y[1] else _neg_fq(y[0])


def f2_sqrt(a):
    """A square root in Fq2 (p = 3 mod 4) or None."""
    if a == (0, 0):
        return (0, 0)
    a1 = bn254.f2_pow(a, (P - 3) // 4)
    alpha = bn254.f2_mul(bn254.f2_sqr(a1), a)
    a0 = bn254.f2_mul(bn254.f2_pow(alpha, P), alpha)
    if a0 == (P - 1, 0):
        return None
    x0 = bn254.f2_mul(a1, a)
    if alpha == (P - 1, 0):
        x = bn254.f2_mul((0, 1), x0)
    else:
        b = bn254.f2_pow(bn254.f2_add((1, 0), alpha), (P - 1) // 2)
        x = bn254.f2_mul(b, x0)
    return x if bn254.f2_sqr(x) == a else None


def g1_from_rng(rng: ChaCha):
    while True:
        x = fq_from_rng(rng)
        greatest = (rng.next_u32() & 1) == 1
        y = bn254.fq_sqrt((x * x * x + 3) % P)
        if y is not None:
            break
    if greatest != _neg_fq(y):
        y = (-y) % P
    return (x, y)


def g2_from_rng(rng: ChaCha):
    while True:
        x = (fq_from_rng(rng), fq_from_rng(rng))
        greatest = (rng.next_u32() & 1) == 1
        y = f2_sqrt(bn254.f2_add(bn254.f2_mul(bn254.f2_sqr(x), x), bn254.B2))
        if y is not None:
            break
    if greatest != _neg_fq2(y):
        y = bn254.f2_neg(y)
    return g2_mul_full((x, y), G2_COFACTOR)


def g2_mul_full(pt, k: int):
    """k * pt with k NOT reduced mod r (bn254.g2_mul reduces: right only inside G2); for clearing
    the twist's cofactor of a point that is not yet in G2."""
    acc = bn254.G2J_INF
    base = bn254.g2j_from_affine(pt)
    while k:
        if k & 1:
            acc = bn254.g2j_add(acc, base)
        base = bn254.g2j_double(base)
        k >>= 1
    return bn254.g2j_to_affine(acc)


def seed_words(h: bytes):
    return [int.from_bytes(h[4 * i:4 * i + 4], "big") for i in range(8)]


def hash_to_g2(transcript: bytes):
    return g2_from_rng(ChaCha(seed_words(transcript)))


def entropy_rng(rand64: bytes, entropy: str) -> ChaCha:
    h = blake2b()
    h.update(rand64)
    h.update(entropy.encode("utf-8"))
    return ChaCha(seed_words(h.digest()))


def beacon_rng(beacon: bytes, num_iterations_exp: int) -> ChaCha:
    return ChaCha(seed_words(beacon_hash(beacon, num_iterations_exp)))


# ------------------------------------------------------------------ contributions

def hash_pubkey(h, c):
    h.update(g1_u(c["deltaAfter"]))
    h.update(g1_u(c["g1_s"]))
    h.update(g1_u(c["g1_sx"]))
    h.update(g2_u(c["g2_spx"]))
    h.update(c["transcript"])


def contribute(z, rng: ChaCha, ctype: int = 0, name: str | None = None, beacon=None):
    """One contribution (zkey contribute: ctype 0; zkey beacon: ctype 1 with beacon = (hash,
    numIterationsExp)) drawn from rng -> the new key (a copy; z.extra["mpc"] must hold the record)."""
    from .setup import contribute_delta
    mpc = z.extra["mpc"]
    th = blake2b()
    th.update(mpc["cs_hash"])
    for c in mpc["contributions"]:
        hash_pubkey(th, c)
    k = fr_from_rng(rng)
    g1_s = g1_from_rng(rng)
    g1_sx = bn254.g1_mul(g1_s, k)
    th.update(g1_u(g1_s))
    th.update(g1_u(g1_sx))
    transcript = th.digest()
    g2_spx = bn254.g2_mul(hash_to_g2(transcript), k)
    out = contribute_delta(z, k)
    c = {"deltaAfter": out.delta1, "g1_s": g1_s, "g1_sx": g1_sx, "g2_spx": g2_spx, "transcript": transcript,
         "type": ctype}
    if name is not None:
        c["name"] = name
    if ctype == 1:
        c["beaconHash"], c["numIterationsExp"] = beacon
    out.extra = dict(z.extra)
    out.extra["mpc"] = {"cs_hash": mpc["cs_hash"], "contributions": list(mpc["contributions"]) + [c]}
    return out, k


def contribute_entropy(z, rand64: bytes, entropy: str, name: str | None = None):
    return contribute(z, entropy_rng(rand64, entropy), 0, name)


def beacon(z, beacon_bytes: bytes, num_iterations_exp: int, name: str | None = None):
    return contribute(z, beacon_rng(beacon_bytes, num_iterations_exp), 1, name,
                      (bytes(beacon_bytes), num_iterations_exp))


# ------------------------------------------------------------------ section 10 bytes

def mpc_name_bytes(name: str) -> bytes:
    """UTF-8 bytes of a contributor name as snarkjs writes them: name.substring(0, 64) counts
    UTF-16 code units (a surrogate pair is two; a cut through one keeps its high half, which
    TextEncoder writes as U+FFFD), then encodes; at most 192 bytes, below the 255 of the length byte."""
    u16 = name.encode("utf-16-le")[:128]
    return u16.decode("utf-16-le", errors="replace").encode("utf-8")


def write_mpc(mpc) -> bytes:
    out = [mpc["cs_hash"], struct.pack("<I", len(mpc["contributions"]))]
    for c in mpc["contributions"]:
        out += [bn254.g1_to_lem(c["deltaAfter"]), bn254.g1_to_lem(c["g1_s"]), bn254.g1_to_lem(c["g1_sx"]),
                bn254.g2_to_lem(c["g2_spx"]), c["transcript"], struct.pack("<I", c.get("type", 0))]
        params = []
        if c.get("name") is not None:
            nm = mpc_name_bytes(c["name"])
            params += [1, len(nm)] + list(nm)
        if c.get("type", 0) == 1:  # id 2 carries its one value byte directly (no length byte)
            params += [2, c["numIterationsExp"], 3, len(c["beaconHash"])] + list(c["beaconHash"])
        out += [struct.pack("<I", len(params)), bytes(params)]
    return b"".join(out)


def read_mpc(sec: bytes):
    cs = bytes(sec[:64])
    (n,) = struct.unpack_from("<I", sec, 64)
    o = 68
    cons = []
    for _ in range(n):
        c = {"deltaAfter": bn254.g1_from_lem(bytes(sec[o:o + 64])), "g1_s": bn254.g1_from_lem(bytes(sec[o + 64:o + 128])),
             "g1_sx": bn254.g1_from_lem(bytes(sec[o + 128:o + 192])),
             "g2_spx": bn254.g2_from_lem(bytes(sec[o + 192:o + 320])), "transcript": bytes(sec[o + 320:o + 384])}
        o += 384
        c["type"], plen = struct.unpack_from("<II", sec, o)
        o += 8
        prm = bytes(sec[o:o + plen])
        o += plen
        j = 0
        while j < len(prm):
            pid = prm[j]
            if pid == 2:  # numIterationsExp: one value byte, no length
                c["numIterationsExp"] = prm[j + 1]
                j += 2
                continue
            if pid not in (1, 3):
                raise ValueError("zkey: MPC parameter %d not recognized" % pid)
            ln = prm[j + 1]
            val = prm[j + 2:j + 2 + ln]
            if pid == 1:
                c["name"] = val.decode("utf-8")
            else:
                c["beaconHash"] = bytes(val)
            j += 2 + ln
        cons.append(c)
    if o != len(sec):
        raise ValueError("zkey: section 10 has trailing bytes")
    return {"cs_hash": cs, "contributions": cons}


# ------------------------------------------------------------------ zkey verify

def same_ratio(g1a, g1b, g2a, g2b) -> bool:
    """e(g1a, g2b) == e(g1b, g2a)."""
    if g1a is None or g1b is None or g2a is None or g2b is None:
        return False
    return bn254.pairing_prod_is_one([(bn254.g1_neg(g1a), g2b), (g1b, g2a)])


def _lincomb_g1(pts, coeffs):
    acc = None
    for p, k in zip(pts, coeffs):
        if p is not None:
            acc = bn254.g1_add(acc, bn254.g1_mul(p, k))
    return acc


def zkey_verify(key: bytes, init: bytes, seed: int = 1) -> tuple[bool, str]:
    """`snarkjs zkey verify` (zkey_verify_frominit.js, recalled) of `key` against `init`, the key
    `zkey new` writes for the same circuit and ptau: the transcript chain of every contribution
    (transcript hash, proof of knowledge g1_s : g1_sx = g2_sp : g2_spx, deltaAfter following the
    previous delta, the beacon's draws), delta1 / delta2 equal to the last deltaAfter, the csHash and
    the unchanged sections equal to the initial key's, and L / H scaled by the same delta^-1
    (random linear combinations, one pairing check each)."""
    from .binfile import read_binfile, read_zkey
    zk = read_zkey(key)
    z0 = read_zkey(init)
    _, secs = read_binfile(key, b"zkey", 1)
    _, secs0 = read_binfile(init, b"zkey", 1)
    sec = lambda b, s, i: b[s[i][0][0]:s[i][0][0] + s[i][0][1]]  # noqa: E731
    mpc = read_mpc(sec(key, secs, 10))
    mpc0 = read_mpc(sec(init, secs0, 10))
    acc = blake2b()
    acc.update(mpc["cs_hash"])
    cur = bn254.G1_GEN
    for i, c in enumerate(mpc["contributions"]):
        th = acc.copy()
        th.update(g1_u(c["g1_s"]))
        th.update(g1_u(c["g1_sx"]))
        if th.digest() != c["transcript"]:
            return False, "INVALID(%d): inconsistent transcript" % i
        g2_sp = hash_to_g2(c["transcript"])
        if not same_ratio(c["g1_s"], c["g1_sx"], g2_sp, c["g2_spx"]):
            return False, "INVALID(%d): public key G1 and G2 do not have the same ratio" % i
        if not same_ratio(cur, c["deltaAfter"], g2_sp, c["g2_spx"]):
            return False, "INVALID(%d): deltaAfter does not follow the public key" % i
        if c["type"] == 1:
            rng = beacon_rng(c["beaconHash"], c["numIterationsExp"])
            k = fr_from_rng(rng)
            g1_s = g1_from_rng(rng)
            if g1_s != c["g1_s"] or bn254.g1_mul(g1_s, k) != c["g1_sx"]:
                return False, "INVALID(%d): does not match the beacon" % i
        hash_pubkey(acc, c)
        cur = c["deltaAfter"]
    for f in ("n_vars", "n_public", "domain_size", "alpha1", "beta1", "beta2", "gamma2"):
        if getattr(zk, f) != getattr(z0, f):
            return False, "INVALID: %s differs from the initial key" % f
    if zk.delta1 != cur:
        return False, "INVALID: delta1 is not the last deltaAfter"
    if not same_ratio(bn254.G1_GEN, cur, bn254.G2_GEN, zk.delta2):
        return False, "INVALID: delta2"
    if mpc["cs_hash"] != mpc0["cs_hash"]:
        return False, "INVALID: circuit does not match (csHash)"
    for s in (3, 4, 5, 6, 7):
        if sec(key, secs, s) != sec(init, secs0, s):
            return False, "INVALID: section %d is not identical to the initial key's" % s
    rnd = random.Random(seed)
    for name, new, old in (("L", zk.c, z0.c), ("H", zk.h, z0.h)):
        if len(new) != len(old):
            return False, "INVALID: %s section size" % name
        co = [rnd.randrange(1, R) for _ in new]
        # e(sum r_i old_i, delta2_init) == e(sum r_i new_i, delta2): new = old delta_init / delta
        if not same_ratio(_lincomb_g1(old, co), _lincomb_g1(new, co), zk.delta2, z0.delta2):
            return False, "INVALID: %s section is not the initial one times delta^-1" % name
    return True, "OK"
