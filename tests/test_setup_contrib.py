"""§8f row 4 (setup acceleration): phase-2 contribution math delta -> k*delta.

CPU: the oracle's restatement keeps the key valid (a proof made with the contributed key
verifies under its verification key, and not under the old one).
GPU: zkp_zkey_contribute is byte-identical to the oracle's contributed key, and the GPU
prover's proofs with it verify."""
import json
import os

import pytest

from oracle import binfile, circuit, groth16, setup
import zkp_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
K = 0x1F2E3D4C5B6A79880123456789ABCDEF00112233445566778899AABBCCDDEEFF % groth16.R


def _case(name):
    zk = open(os.path.join(GOLD, "circuit_%s.zkey" % name), "rb").read()
    wt = open(os.path.join(GOLD, "circuit_%s.wtns" % name), "rb").read()
    return zk, wt


def test_oracle_contribution_keeps_key_valid():
    zk, wt = _case("tiny")
    z = binfile.read_zkey(zk)
    z2 = setup.contribute_delta(z, K)
    w = binfile.read_wtns(wt)[1]
    proof, pub = groth16.prove(z2, w, 5, 7)
    assert groth16.verify_with_zkey(z2, pub, proof)
    assert not groth16.verify_with_zkey(z, pub, proof)
    with pytest.raises(ValueError):
        setup.contribute_delta(z, groth16.R)


@pytest.mark.gpu
@pytest.mark.parametrize("name,k", [("tiny", K), ("small", K), ("small", 1), ("venmo_mini", K + groth16.R)])
def test_gpu_contribute_matches_oracle_and_proves(name, k):
    zk, wt = _case(name)
    out = zkp_amd.zkey_contribute(zk, k)
    z2 = setup.contribute_delta(binfile.read_zkey(zk), k)
    assert out == binfile.write_zkey(z2)
    if name != "tiny":
        (a, b, c), pub = zkp_amd.Prover(out).prove_raw(wt)
        assert groth16.verify_with_zkey(z2, pub, {"A": a, "B": b, "C": c})


@pytest.mark.gpu
def test_gpu_contribute_rejects_zero():
    zk, _ = _case("tiny")
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.zkey_contribute(zk, groth16.R)
    assert e.value.status == 1
