"""snarkjs binary containers (.zkey v1 groth16, .wtns v2) — TEST INFRASTRUCTURE ONLY.

Restates binfileutils 0.0.11 / fastfile 0.0.20 + snarkjs ``zkey_utils`` /
``wtns_utils`` layouts (upstream pins reference ``package-lock.json:454-456,
2054-2058``; SURVEY.md App. A, recalled upstream layout, unpinned offline).

Container: 4-byte magic, u32 version, u32 nSections, then per section
``u32 id, u64 byteLength, payload``; all little-endian.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

from . import bn254

ZKEY_GROTH16 = 1


def write_binfile(magic: bytes, version: int, sections) -> bytes:
    """sections: list of (id, payload bytes) in file order."""
    out = [magic, struct.pack("<II", version, len(sections))]
    for sid, payload in sections:
        out.append(struct.pack("<IQ", sid, len(payload)))
        out.append(payload)
    return b"".join(out)


def read_binfile(buf: bytes, magic: bytes, max_version: int):
    if len(buf) < 12 or buf[:4] != magic:
        raise ValueError("%s: invalid file format" % magic.decode())
    version, nsec = struct.unpack_from("<II", buf, 4)
    if version > max_version:
        raise ValueError("%s: version not supported" % magic.decode())
    pos = 12
    sections = {}
    for _ in range(nsec):
        sid, ln = struct.unpack_from("<IQ", buf, pos)
        pos += 12
        if pos + ln > len(buf):
            raise ValueError("%s: truncated section %d" % (magic.decode(), sid))
        sections.setdefault(sid, []).append((pos, ln))
        pos += ln
    return version, sections


# ------------------------------------------------------------------ wtns


def write_wtns(witness) -> bytes:
    n8 = 32
    sec1 = struct.pack("<I", n8) + bn254.int_to_le(bn254.R) + struct.pack("<I", len(witness))
    sec2 = b"".join(bn254.int_to_le(w % bn254.R) for w in witness)
    return write_binfile(b"wtns", 2, [(1, sec1), (2, sec2)])


def read_wtns(buf: bytes):
    _, secs = read_binfile(buf, b"wtns", 2)
    p1, _ = secs[1][0]
    (n8,) = struct.unpack_from("<I", buf, p1)
    q = bn254.le_to_int(buf[p1 + 4:p1 + 4 + n8])
    (nw,) = struct.unpack_from("<I", buf, p1 + 4 + n8)
    p2, ln2 = secs[2][0]
    if ln2 != nw * n8:
        raise ValueError("wtns: invalid witness section size")
    w = [bn254.le_to_int(buf[p2 + i * n8:p2 + (i + 1) * n8]) for i in range(nw)]
    return q, w


# ------------------------------------------------------------------ r1cs / ptau (setup inputs)


def write_r1cs(r1cs) -> bytes:
    """circom ``.r1cs`` v1 (binfile "r1cs"; read by snarkjs ``zkey new`` through the r1csfile
    package, reference call site dizkus-scripts/3_gen_chunk_zkey.sh:18; recalled layout,
    unpinned offline): section 1 header (u32 n8, prime r, u32 nWires, u32 nPubOut, u32 nPubIn,
    u32 nPrvIn, u64 nLabels, u32 nConstraints), section 2 the constraints (A, B, C linear
    combinations: u32 count, then count x (u32 wire, n8-byte LE coefficient)), section 3 the
    wire -> label map (u64 per wire).  All public signals are written as public inputs."""
    n8 = 32
    npub = r1cs.n_public
    sec1 = (struct.pack("<I", n8) + bn254.int_to_le(bn254.R) +
            struct.pack("<IIII", r1cs.n_vars, 0, npub, r1cs.n_vars - 1 - npub) +
            struct.pack("<QI", r1cs.n_vars, r1cs.n_constraints))
    parts = []
    for lcs in r1cs.constraints:
        for lc in lcs:
            parts.append(struct.pack("<I", len(lc)))
            for sig, v in lc:
                parts.append(struct.pack("<I", sig) + bn254.int_to_le(v % bn254.R))
    sec3 = b"".join(struct.pack("<Q", i) for i in range(r1cs.n_vars))
    return write_binfile(b"r1cs", 1, [(1, sec1), (2, b"".join(parts)), (3, sec3)])


def write_ptau(power: int, tau_g1, tau_g2, alpha_tau_g1, beta_tau_g1, beta_g2, l_tau_g1, l_tau_g2,
               l_alpha_tau_g1, l_beta_tau_g1) -> bytes:
    """snarkjs ``.ptau`` v1 after ``powersoftau prepare phase2`` (recalled layout, unpinned
    offline): 1 header (u32 n8, prime q, u32 power, u32 ceremonyPower), 2 tauG1 (2^(power+1)-1
    points), 3 tauG2 (2^power), 4 alphaTauG1, 5 betaTauG1 (2^power each), 6 betaG2, 7 the
    contributions (u32 count = 0), 12..15 the Lagrange forms lTauG1, lTauG2, lAlphaTauG1,
    lBetaTauG1 of every level p = 0..power concatenated (level p = 2^p points at 2^p - 1)."""
    g1 = lambda pts: b"".join(bn254.g1_to_lem(p) for p in pts)
    g2 = lambda pts: b"".join(bn254.g2_to_lem(p) for p in pts)
    sec1 = struct.pack("<I", 32) + bn254.int_to_le(bn254.P) + struct.pack("<II", power, power)
    return write_binfile(b"ptau", 1, [
        (1, sec1), (2, g1(tau_g1)), (3, g2(tau_g2)), (4, g1(alpha_tau_g1)), (5, g1(beta_tau_g1)),
        (6, g2([beta_g2])), (7, struct.pack("<I", 0)),
        (12, g1(l_tau_g1)), (13, g2(l_tau_g2)), (14, g1(l_alpha_tau_g1)), (15, g1(l_beta_tau_g1))])


# ------------------------------------------------------------------ zkey


@dataclass
class ZKey:
    n_vars: int
    n_public: int
    domain_size: int
    alpha1: tuple
    beta1: tuple
    beta2: tuple
    gamma2: tuple
    delta1: tuple
    delta2: tuple
    ic: list
    coefs: list  # (matrix, constraint, signal, value) with value = plain coefficient (not *R^2)
    a: list
    b1: list
    b2: list
    c: list  # length n_vars - n_public - 1
    h: list  # length domain_size
    extra: dict = field(default_factory=dict)


def write_zkey(z: ZKey) -> bytes:
    R = bn254.R
    R2 = (bn254.MONT_R * bn254.MONT_R) % R
    sec1 = struct.pack("<I", ZKEY_GROTH16)
    sec2 = b"".join([
        struct.pack("<I", 32), bn254.int_to_le(bn254.P),
        struct.pack("<I", 32), bn254.int_to_le(R),
        struct.pack("<III", z.n_vars, z.n_public, z.domain_size),
        bn254.g1_to_lem(z.alpha1), bn254.g1_to_lem(z.beta1), bn254.g2_to_lem(z.beta2),
        bn254.g2_to_lem(z.gamma2), bn254.g1_to_lem(z.delta1), bn254.g2_to_lem(z.delta2),
    ])
    sec3 = b"".join(bn254.g1_to_lem(p) for p in z.ic)
    parts = [struct.pack("<I", len(z.coefs))]
    for m, c, s, v in z.coefs:
        parts.append(struct.pack("<III", m, c, s))
        parts.append(bn254.int_to_le(v % R * R2 % R))
    sec4 = b"".join(parts)
    sec5 = b"".join(bn254.g1_to_lem(p) for p in z.a)
    sec6 = b"".join(bn254.g1_to_lem(p) for p in z.b1)
    sec7 = b"".join(bn254.g2_to_lem(p) for p in z.b2)
    sec8 = b"".join(bn254.g1_to_lem(p) for p in z.c)
    sec9 = b"".join(bn254.g1_to_lem(p) for p in z.h)
    # section 10, the MPC record (prove ignores it): z.extra["mpc"] (oracle/mpc.py) when the key
    # carries one, else a zero csHash and no contributions
    mpc = z.extra.get("mpc")
    if mpc is not None:
        from .mpc import write_mpc
        sec10 = write_mpc(mpc)
    else:
        sec10 = bytes(64) + struct.pack("<I", 0)
    return write_binfile(b"zkey", 1, [(1, sec1), (2, sec2), (3, sec3), (4, sec4), (5, sec5),
                                      (6, sec6), (7, sec7), (8, sec8), (9, sec9), (10, sec10)])


def read_zkey(buf: bytes) -> ZKey:
    R = bn254.R
    R2inv = bn254.inv((bn254.MONT_R * bn254.MONT_R) % R, R)
    _, secs = read_binfile(buf, b"zkey", 1)
    p1, _ = secs[1][0]
    (proto,) = struct.unpack_from("<I", buf, p1)
    if proto != ZKEY_GROTH16:
        raise ValueError("zkey file is not groth16")
    o, _ = secs[2][0]
    (n8q,) = struct.unpack_from("<I", buf, o)
    o += 4
    q = bn254.le_to_int(buf[o:o + n8q])
    o += n8q
    (n8r,) = struct.unpack_from("<I", buf, o)
    o += 4
    r = bn254.le_to_int(buf[o:o + n8r])
    o += n8r
    if q != bn254.P or r != bn254.R:
        raise ValueError("zkey curve not supported")
    n_vars, n_public, domain = struct.unpack_from("<III", buf, o)
    o += 12

    def g1(off):
        return bn254.g1_from_lem(buf[off:off + 64]), off + 64

    def g2(off):
        return bn254.g2_from_lem(buf[off:off + 128]), off + 128

    alpha1, o = g1(o)
    beta1, o = g1(o)
    beta2, o = g2(o)
    gamma2, o = g2(o)
    delta1, o = g1(o)
    delta2, o = g2(o)

    def g1s(sid, n):
        off, ln = secs[sid][0]
        if ln != 64 * n:
            raise ValueError("zkey: section %d has wrong size" % sid)
        return [bn254.g1_from_lem(buf[off + 64 * i:off + 64 * (i + 1)]) for i in range(n)]

    ic = g1s(3, n_public + 1)
    off, _ = secs[4][0]
    (ncoef,) = struct.unpack_from("<I", buf, off)
    off += 4
    coefs = []
    for _ in range(ncoef):
        m, c, s = struct.unpack_from("<III", buf, off)
        v = bn254.le_to_int(buf[off + 12:off + 44]) * R2inv % R
        coefs.append((m, c, s, v))
        off += 44
    a = g1s(5, n_vars)
    b1 = g1s(6, n_vars)
    off7, ln7 = secs[7][0]
    if ln7 != 128 * n_vars:
        raise ValueError("zkey: section 7 has wrong size")
    b2 = [bn254.g2_from_lem(buf[off7 + 128 * i:off7 + 128 * (i + 1)]) for i in range(n_vars)]
    c = g1s(8, n_vars - n_public - 1)
    h = g1s(9, domain)
    z = ZKey(n_vars, n_public, domain, alpha1, beta1, beta2, gamma2, delta1, delta2, ic, coefs,
             a, b1, b2, c, h)
    if 10 in secs:
        from .mpc import read_mpc
        off, ln = secs[10][0]
        z.extra["mpc"] = read_mpc(buf[off:off + ln])
    return z


def read_zkey_vk(buf):
    """Only what verification needs (header points + IC, section 3) from a zkey buffer
    (bytes or a memoryview over a multi-GB key: nothing else is touched)."""
    _, secs = read_binfile(buf, b"zkey", 1)
    o, _ = secs[2][0]
    o += 4 + 32 + 4 + 32
    n_vars, n_public, domain = struct.unpack_from("<III", buf, o)
    o += 12
    rd1 = lambda off: bn254.g1_from_lem(bytes(buf[off:off + 64]))
    rd2 = lambda off: bn254.g2_from_lem(bytes(buf[off:off + 128]))
    alpha1, beta1, beta2 = rd1(o), rd1(o + 64), rd2(o + 128)
    gamma2, delta1, delta2 = rd2(o + 256), rd1(o + 384), rd2(o + 448)
    off, ln = secs[3][0]
    if ln != 64 * (n_public + 1):
        raise ValueError("zkey: section 3 has wrong size")
    ic = [rd1(off + 64 * i) for i in range(n_public + 1)]
    return {"n_vars": n_vars, "n_public": n_public, "domain": domain, "alpha1": alpha1, "beta1": beta1,
            "beta2": beta2, "gamma2": gamma2, "delta1": delta1, "delta2": delta2, "ic": ic}
