"""GPU parity of the kernel-level entry points (MSM G1/G2, NTT, quotient) against
the oracle's golden vectors — bit-exact (integer arithmetic)."""
import json
import os

import pytest

from oracle import bn254, circuit, groth16, ntt
import zkp_amd

pytestmark = pytest.mark.gpu
R = bn254.R


def _load_msm(golden_dir, name, n, g2):
    blob = open(os.path.join(golden_dir, name), "rb").read()
    pw = 128 if g2 else 64
    pts = blob[: n * pw]
    scal = blob[n * pw: n * pw + n * 32]
    exp = blob[n * pw + n * 32:]
    return pts, scal, exp


@pytest.mark.parametrize("n", [64, 1024])
def test_msm_g1_golden(golden_dir, n):
    pts, scal, exp = _load_msm(golden_dir, "msm_g1_%d.bin" % n, n, False)
    got = zkp_amd.msm_g1(pts, scal)
    want = None if not any(exp) else (bn254.le_to_int(exp[:32]), bn254.le_to_int(exp[32:]))
    assert got == want


@pytest.mark.parametrize("n", [64, 256])
def test_msm_g2_golden(golden_dir, n):
    pts, scal, exp = _load_msm(golden_dir, "msm_g2_%d.bin" % n, n, True)
    got = zkp_amd.msm_g2(pts, scal)
    v = [bn254.le_to_int(exp[32 * i:32 * i + 32]) for i in range(4)]
    want = None if not any(exp) else ((v[0], v[1]), (v[2], v[3]))
    assert got == want


def _pts(n, seed):
    rng = circuit.SplitMix64(seed, 0)
    g = bn254.FixedBase(bn254.G1_GEN)
    return [g.mul(rng.fr() or 1) for _ in range(n)]


def _blob(pts, scal):
    return b"".join(bn254.g1_to_lem(p) for p in pts), b"".join(bn254.int_to_le(x) for x in scal)


def _plan(monkeypatch, dense):
    monkeypatch.setenv("ZKP_MSM", "plan=" + ("dense" if dense in (1, "1") else "compact"))


@pytest.mark.parametrize("dense", ["1", "0"])  # kernel-level default (dense plan) and the witness plan's variant
def test_msm_g1_edge_distributions(monkeypatch, dense):
    _plan(monkeypatch, dense)
    pts = _pts(300, 99)
    cases = {
        "empty": ([], []),
        "single_zero": (pts[:1], [0]),
        "all_zero": (pts, [0] * 300),
        "all_one": (pts, [1] * 300),            # every point in ONE bucket (circuit-like)
        "same_scalar": (pts, [12345678901234567] * 300),
        "same_point": ([pts[0]] * 300, list(range(1, 301))),  # doubling inside buckets
        "above_r": (pts[:8], [R + 5, 2 * R + 1, (1 << 256) - 1, R, R - 1, 1, 2, 3]),
        "bytes": (pts, [(i * 37) % 256 for i in range(300)]),
    }
    for name, (p, s) in cases.items():
        pb, sb = _blob(p, s)
        got = zkp_amd.msm_g1(pb, sb)
        want = groth16.msm_g1(p, [x % R for x in s])
        assert got == want, name


@pytest.mark.parametrize("dense", ["1", "0"])
def test_msm_g1_skewed_and_multigroup(monkeypatch, dense):
    # skewed (one bucket), uniform, sparse and multi-group inputs on both plan variants: the
    # wave-aggregated LDS claims and the tiled pass C (compact), one workgroup per sub-bin (dense)
    _plan(monkeypatch, dense)
    pts = _pts(300, 41)
    rng = circuit.SplitMix64(42, 1)
    uni = [rng.fr() for _ in range(300)]
    cases = [
        (pts, uni, 0, 0),
        (pts, [1] * 150 + uni[:150], 0, 0),          # circuit-like: half the entries in bucket 0
        (pts, [1] * 300, 8, 0),
        (pts, uni, 8, 4),                             # 8 bucket groups
        (pts, [0] * 299 + [5], 0, 0),
        (pts[:1], [0], 0, 0),
    ]
    for p, s, c, d in cases:
        pb, sb = _blob(p, s)
        assert zkp_amd.msm_g1(pb, sb, window_bits=c, table_depth=d) == groth16.msm_g1(p, s), (c, d)


def test_msm_g1_dense_counting_sort(monkeypatch):
    # the dense plan grouped by the hand-written three-pass bucket sort: uniform, skewed (one
    # bucket), sparse, degenerate, multi-group and every-window-bits inputs against the oracle
    _plan(monkeypatch, 1)
    pts = _pts(300, 43)
    rng = circuit.SplitMix64(44, 1)
    uni = [rng.fr() for _ in range(300)]
    cases = [
        (pts, uni, 0, 0),
        (pts, uni, 20, 0),                            # the H plan's window bits: 2^19 buckets, fine bits 10
        (pts, uni, 24, 0),                            # fine bits 14 (the largest LDS histogram)
        (pts, uni, 8, 0), (pts, uni, 9, 0),           # W = 32 / 29 windows: one scalar per thread per round
        (pts, uni, 10, 4),                            # 7 bucket groups (bucket count not a power of two)
        (pts, [1] * 150 + uni[:150], 0, 0),           # half the entries in one bucket
        (pts, [1] * 300, 16, 0),
        ([pts[0]] * 300, list(range(1, 301)), 0, 0),  # doublings inside buckets
        (pts, [0] * 299 + [5], 0, 0),
        (pts, [0] * 300, 0, 0),
        (pts[:1], [0], 0, 0),
        (pts[:8], [R + 5, 2 * R + 1, (1 << 256) - 1, R, R - 1, 1, 2, 3], 0, 0),
    ]
    for p, s, c, d in cases:
        pb, sb = _blob(p, s)
        assert zkp_amd.msm_g1(pb, sb, window_bits=c, table_depth=d) == groth16.msm_g1(p, [x % R for x in s]), (c, d)


@pytest.mark.parametrize("c", [17, 18, 19, 20, 21, 22])
def test_msm_dense_window_bits(monkeypatch, c):
    # the hand-written sort's bin / sub-bin / bucket bit splits of every window width around the
    # prover's choices (c = 18: 6 + 6 + 5 bits, 19: 7 + 6 + 5, 21: 8 + 7 + 5 ...), 2^15 uniform
    # scalars over 64 bases: dense plan == compacted plan == the oracle's sum
    rng = circuit.SplitMix64(46, 1)
    n = 1 << 15
    g = bn254.FixedBase(bn254.G1_GEN)
    base = [g.mul(rng.fr() or 1) for _ in range(64)]
    pts = [base[i % 64] for i in range(n)]
    sc = [rng.fr() for _ in range(n)]
    pb, sb = _blob(pts, sc)
    _plan(monkeypatch, 1)
    got = zkp_amd.msm_g1(pb, sb, window_bits=c)
    _plan(monkeypatch, 0)
    assert zkp_amd.msm_g1(pb, sb, window_bits=c) == got
    acc = [0] * 64
    for i, x in enumerate(sc):
        acc[i % 64] = (acc[i % 64] + x) % R
    assert got == groth16.msm_g1(base, acc)


def test_msm_dense_counting_sort_large(monkeypatch):
    # several scatter workgroups and every coarse bin populated: 2^14 uniform scalars at c = 20 on
    # the dense plan vs the compacted plan of the same input; the subset sums (c = 20: 18 sums of
    # 2^16 values) take the chain level below the trees, c = 13 the trees from the inputs
    rng = circuit.SplitMix64(45, 1)
    n = 1 << 14
    g = bn254.FixedBase(bn254.G1_GEN)
    base = [g.mul(rng.fr() or 1) for _ in range(64)]
    pts = [base[i % 64] for i in range(n)]
    sc = [rng.fr() for _ in range(n)]
    pb, sb = _blob(pts, sc)
    _plan(monkeypatch, 0)
    want = zkp_amd.msm_g1(pb, sb, window_bits=20)
    _plan(monkeypatch, 1)
    assert zkp_amd.msm_g1(pb, sb, window_bits=20) == want
    assert zkp_amd.msm_g1(pb, sb, window_bits=13) == want
    # the oracle on the same sum: scalars of equal bases add up
    acc = [0] * 64
    for i, x in enumerate(sc):
        acc[i % 64] = (acc[i % 64] + x) % R
    assert want == groth16.msm_g1(base, acc)


@pytest.mark.parametrize("k", [1, 4, 10, 12])
def test_ntt_golden(golden_dir, k):
    d = json.load(open(os.path.join(golden_dir, "ntt_%d.json" % k)))
    a = [int(x) for x in d["input"]]
    assert zkp_amd.ntt_fr(a, 0) == [int(x) for x in d["forward"]]
    assert zkp_amd.ntt_fr(a, 1) == [int(x) for x in d["inverse"]]
    assert zkp_amd.ntt_fr(a, 2) == [int(x) for x in d["coset"]]


@pytest.mark.parametrize("k", [2, 3, 5, 6, 7, 8, 9, 11, 13, 15])
def test_ntt_every_pass_geometry(k):
    """Forward, inverse and coset extension against the oracle's radix-2 NTT for pass splits with odd
    and even pass widths (3: b = 3; 5, 7: one odd pass; 9 = 5 + 4; 11 = 6 + 5; 13 = 7 + 6; 15 = 8 + 7) and
    tiles smaller than 1024 elements: the odd pass's radix-2 stage runs first and every DFT's last
    radix-4 pair skips its w^0 product (ntt.hip, round 5)"""
    rng = circuit.SplitMix64(100 + k, 3)
    a = [rng.fr() for _ in range(1 << k)]
    assert zkp_amd.ntt_fr(a, 0) == ntt.fft(a)
    inv_a = ntt.ifft(a)
    assert zkp_amd.ntt_fr(a, 1) == inv_a
    assert zkp_amd.ntt_fr(a, 2) == ntt.fft(ntt.batch_apply_key(inv_a, 1, ntt.coset_gen(1 << k)))


@pytest.mark.parametrize("k", [14, 17, 20])
def test_ntt_roundtrip_large(k):
    rng = circuit.SplitMix64(k, 2)
    a = [rng.fr() for _ in range(1 << k)]
    fwd = zkp_amd.ntt_fr(a, 0)
    assert zkp_amd.ntt_fr(fwd, 1) == a
    # spot-check a few outputs against the naive DFT definition
    w = ntt.ROOTS[k]
    for j in (0, 1, 12345 % (1 << k), (1 << k) - 1):
        wj, cur, acc = pow(w, j, R), 1, 0
        for x in a:
            acc += x * cur
            cur = cur * wj % R
        assert fwd[j] == acc % R


@pytest.mark.parametrize("name", ["tiny", "small", "venmo_mini"])
def test_quotient_golden(golden_dir, name):
    zk = open(os.path.join(golden_dir, "circuit_%s.zkey" % name), "rb").read()
    wt = open(os.path.join(golden_dir, "circuit_%s.wtns" % name), "rb").read()
    q = open(os.path.join(golden_dir, "quotient_%s.bin" % name), "rb").read()
    p = zkp_amd.Prover(zk)
    want = [bn254.le_to_int(q[32 * i:32 * i + 32]) for i in range(len(q) // 32)]
    assert p.quotient(wt) == want


# Pippenger parameter variants: window bits c and base-table depth T (T = W: one shared
# bucket set over precomputed 2^(c t) P rows; T = 1: one bucket group per window;
# 1 < T < W: several groups folded by Horner with shift c*T).  Bit-exact vs the oracle.
# (22, 2): 6 groups of 2^21 buckets = 24 key bits, the sort's 6-bit tiled pass C; (23, 2): 6 groups of
# 2^22 buckets = 25 key bits; (24, 1): 11 groups of 2^23 buckets = 27 key bits, the largest the sort
# takes (b3 = 9).
@pytest.mark.parametrize("dense", ["1", "0"])
@pytest.mark.parametrize("c,depth", [(0, 1), (8, 0), (8, 3), (9, 7), (13, 0), (20, 0), (24, 0), (22, 2), (23, 2),
                                     (24, 1)])
def test_msm_g1_params(monkeypatch, c, depth, dense):
    _plan(monkeypatch, dense)
    pts = _pts(200, 5)
    rng = circuit.SplitMix64(6, 1)
    sc = [rng.fr() for _ in range(200)]
    pb, sb = _blob(pts, sc)
    assert zkp_amd.msm_g1(pb, sb, window_bits=c, table_depth=depth) == groth16.msm_g1(pts, sc)


@pytest.mark.parametrize("c", [5, 25])
def test_msm_window_bits_out_of_range(c):
    pts = _pts(4, 5)
    pb, sb = _blob(pts, [1, 2, 3, 4])
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.msm_g1(pb, sb, window_bits=c)
    assert e.value.status == 1 and "window bits" in e.value.message


def test_msm_g1_every_digit_one():
    # every window digit of every scalar is 1 -> all n*W entries land in ONE bucket of the
    # shared set: exercises the heavy-bucket merge levels
    pts = _pts(200, 8)
    s = sum(1 << (8 * w) for w in range(31))
    pb, sb = _blob(pts, [s] * 200)
    assert zkp_amd.msm_g1(pb, sb, window_bits=8) == groth16.msm_g1(pts, [s % R] * 200)


@pytest.mark.parametrize("c,depth", [(0, 1), (8, 0), (8, 4)])
def test_msm_g2_params(golden_dir, c, depth):
    n = 64
    pts, scal, exp = _load_msm(golden_dir, "msm_g2_%d.bin" % n, n, True)
    v = [bn254.le_to_int(exp[32 * i:32 * i + 32]) for i in range(4)]
    want = None if not any(exp) else ((v[0], v[1]), (v[2], v[3]))
    assert zkp_amd.msm_g2(pts, scal, window_bits=c, table_depth=depth) == want
