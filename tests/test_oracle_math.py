"""Self-consistency of the CPU oracle and its golden fixtures."""
import hashlib
import json
import os

import pytest

from oracle import binfile, bn254, circuit, groth16, ntt, setup

R = bn254.R
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_roots_of_unity():
    assert ntt.NQR == 5
    assert pow(ntt.ROOTS[28], 1 << 28, R) == 1 and pow(ntt.ROOTS[28], 1 << 27, R) == R - 1
    for k in range(28):
        assert ntt.ROOTS[k] == ntt.ROOTS[k + 1] ** 2 % R


@pytest.mark.parametrize("k", [0, 1, 3, 6])
def test_fft_matches_definition(k):
    rng = circuit.SplitMix64(k, 2)
    a = [rng.fr() for _ in range(1 << k)]
    assert ntt.fft(a) == ntt.naive_dft(a, ntt.ROOTS[k])
    assert ntt.ifft(ntt.fft(a)) == a


def test_coset_extension_is_evaluation_on_coset():
    rng = circuit.SplitMix64(9, 2)
    n = 16
    vals = [rng.fr() for _ in range(n)]
    coef = ntt.ifft(vals)
    g = ntt.coset_gen(n)
    out = ntt.fft(ntt.batch_apply_key(coef, 1, g))
    w = ntt.ROOTS[4]
    for j in (0, 5, 15):
        x = g * pow(w, j, R) % R
        assert out[j] == sum(c * pow(x, i, R) for i, c in enumerate(coef)) % R


def test_bilinearity_and_order():
    P, Q = bn254.G1_GEN, bn254.G2_GEN
    e = bn254.pairing(P, Q)
    assert e != bn254.F12_ONE
    assert bn254.pairing(bn254.g1_mul(P, 6), Q) == bn254.pairing(bn254.g1_mul(P, 2), bn254.g2_mul(Q, 3))
    assert bn254.f12_pow(e, R) == bn254.F12_ONE


def test_manifest_hashes():
    man = json.load(open(os.path.join(GOLD, "manifest.json")))
    for f, h in man["sha256"].items():
        assert hashlib.sha256(open(os.path.join(GOLD, f), "rb").read()).hexdigest() == h, f


@pytest.mark.parametrize("name", ["tiny", "small", "venmo_mini"])
def test_golden_proofs_verify(name):
    z = binfile.read_zkey(open(os.path.join(GOLD, "circuit_%s.zkey" % name), "rb").read())
    _, w = binfile.read_wtns(open(os.path.join(GOLD, "circuit_%s.wtns" % name), "rb").read())
    proof = groth16.proof_from_json_obj(json.load(open(os.path.join(GOLD, "proof_%s.json" % name))))
    pub = [int(x) for x in json.load(open(os.path.join(GOLD, "public_%s.json" % name)))]
    assert pub == w[1:z.n_public + 1]
    assert groth16.verify_with_zkey(z, pub, proof)
    vk = json.load(open(os.path.join(GOLD, "vkey_%s.json" % name)))
    assert vk["vk_alphabeta_12"] == bn254.f12_to_obj(bn254.pairing_snarkjs(z.alpha1, z.beta2))
    bad = dict(proof)
    bad["C"] = bn254.g1_add(proof["C"], bn254.G1_GEN)
    assert not groth16.verify_with_zkey(z, pub, bad)


def test_tiny_regenerates_bit_exactly():
    man = json.load(open(os.path.join(GOLD, "manifest.json")))["circuits"]["tiny"]
    r1cs, w = circuit.gen_circuit(man["n_vars"], man["n_constraints"], man["n_public"], man["circuit_seed"])
    assert circuit.check_witness(r1cs, w)
    zb = binfile.write_zkey(setup.setup(r1cs, man["setup_seed"]))
    assert zb == open(os.path.join(GOLD, "circuit_tiny.zkey"), "rb").read()
    z = binfile.read_zkey(zb)
    proof, pub = groth16.prove(z, w, int(man["r"]), int(man["s"]))
    assert groth16.js_stringify(groth16.proof_to_json_obj(proof)) == open(os.path.join(GOLD, "proof_tiny.json")).read()


def test_quotient_golden_small():
    z = binfile.read_zkey(open(os.path.join(GOLD, "circuit_small.zkey"), "rb").read())
    _, w = binfile.read_wtns(open(os.path.join(GOLD, "circuit_small.wtns"), "rb").read())
    q = open(os.path.join(GOLD, "quotient_small.bin"), "rb").read()
    assert groth16.quotient_scalars(z, w) == [bn254.le_to_int(q[32 * i:32 * i + 32]) for i in range(len(q) // 32)]


def test_wtns_zkey_roundtrip_and_errors():
    r1cs, w = circuit.gen_circuit(40, 45, 3, 5)
    z = setup.setup(r1cs, 6)
    zb = binfile.write_zkey(z)
    z2 = binfile.read_zkey(zb)
    assert (z2.a, z2.b2, z2.h, z2.coefs) == (z.a, z.b2, z.h, z.coefs)
    q, w2 = binfile.read_wtns(binfile.write_wtns(w))
    assert q == R and w2 == [x % R for x in w]
    with pytest.raises(ValueError):
        binfile.read_zkey(b"xkey" + zb[4:])


def test_read_zkey_vk_matches_full_reader(golden_dir):
    """The header-only reader the full-size GPU tests verify with (memoryview over a multi-GB
    key) returns the full reader's verification key."""
    from oracle import binfile
    buf = open(os.path.join(golden_dir, "circuit_small.zkey"), "rb").read()
    z = binfile.read_zkey(buf)
    vk = binfile.read_zkey_vk(memoryview(buf))
    assert (vk["alpha1"], vk["beta2"], vk["gamma2"], vk["delta2"], vk["ic"]) == (z.alpha1, z.beta2, z.gamma2,
                                                                                 z.delta2, z.ic)
    assert (vk["n_vars"], vk["n_public"], vk["domain"]) == (z.n_vars, z.n_public, z.domain_size)
