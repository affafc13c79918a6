"""The host pairing behind verify-before-return (csrc/host_pairing.cpp; SURVEY.md §5, the
reference verifies every proof after proving: dizkus-scripts/5_gen_proof.sh:14-21) -- CPU only,
no GPU: pinned by the reference's own GT value and checked against the oracle.

* zkp_pairing(vk_alpha_1, vk_beta_2) == vk_alphabeta_12 of reference app/src/helpers/vkey.ts:52-82
  (snarkjs' final-exponentiation convention), and bilinearity e(aP, bQ) == e(abP, Q).
* zkp_proof_verify accepts every golden proof under its zkey's verification key and rejects a
  proof with a changed public signal, a swapped coordinate, a signal >= r (Verifier.sol:347) and
  a B point off the subgroup-checked twist; it agrees with the oracle's restated Verifier.sol.
"""
import json
import os

import pytest

from oracle import binfile, bn254, groth16
import zkp_amd

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_fixtures.json")))
VK = FIX["vkey_ts"]


def _g2(o):
    return ((int(o[0][0]), int(o[0][1])), (int(o[1][0]), int(o[1][1])))


def test_pairing_reproduces_vk_alphabeta_12():
    a1 = (int(VK["vk_alpha_1"][0]), int(VK["vk_alpha_1"][1]))
    got = zkp_amd.pairing(a1, _g2(VK["vk_beta_2"]))
    assert [[[str(x[0]), str(x[1])] for x in c] for c in got] == VK["vk_alphabeta_12"]


def test_pairing_bilinear_and_matches_oracle():
    p, q = bn254.g1_mul(bn254.G1_GEN, 7), bn254.g2_mul(bn254.G2_GEN, 11)
    e1 = zkp_amd.pairing(bn254.g1_mul(p, 5), bn254.g2_mul(q, 3))
    e2 = zkp_amd.pairing(bn254.g1_mul(p, 15), q)
    assert e1 == e2
    want = bn254.pairing_snarkjs(p, q)
    assert zkp_amd.pairing(p, q) == [list(c) for c in want]
    one = [[(1, 0), (0, 0), (0, 0)], [(0, 0), (0, 0), (0, 0)]]
    assert zkp_amd.pairing(None, q) == one


def _case(golden_dir, name):
    zk = open(os.path.join(golden_dir, "circuit_%s.zkey" % name), "rb").read()
    proof = json.load(open(os.path.join(golden_dir, "proof_%s.json" % name)))
    pub = [int(x) for x in json.load(open(os.path.join(golden_dir, "public_%s.json" % name)))]
    a = (int(proof["pi_a"][0]), int(proof["pi_a"][1]))
    b = ((int(proof["pi_b"][0][0]), int(proof["pi_b"][0][1])), (int(proof["pi_b"][1][0]), int(proof["pi_b"][1][1])))
    c = (int(proof["pi_c"][0]), int(proof["pi_c"][1]))
    return zk, (a, b, c), pub


@pytest.mark.parametrize("name", ["tiny", "small", "venmo_mini"])
def test_proof_verify_golden_and_tampered(golden_dir, name):
    zk, (a, b, c), pub = _case(golden_dir, name)
    assert zkp_amd.proof_verify(zk, (a, b, c), pub)
    z = binfile.read_zkey(zk)
    assert groth16.verify_with_zkey(z, pub, {"A": a, "B": b, "C": c})
    if pub:
        bad = list(pub)
        bad[0] = (bad[0] + 1) % bn254.R
        assert not zkp_amd.proof_verify(zk, (a, b, c), bad)
        over = list(pub)
        over[0] = pub[0] + bn254.R  # same residue, but >= r: Verifier.sol:347 rejects it
        assert not zkp_amd.proof_verify(zk, (a, b, c), over)
    assert not zkp_amd.proof_verify(zk, (c, b, a), pub)
    assert not zkp_amd.proof_verify(zk, (a, b, bn254.g1_add(c, bn254.G1_GEN)), pub)
    assert not zkp_amd.proof_verify(zk, (a, (b[0], bn254.f2_neg(b[1])), c), pub)
