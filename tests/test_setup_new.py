"""§8f row 4 (setup acceleration): `snarkjs zkey new <circuit.r1cs> <pot.ptau>` (reference
dizkus-scripts/3_gen_chunk_zkey.sh:18).

The ptau and r1cs layouts are restated (oracle/binfile.py write_ptau / write_r1cs; recalled,
"parity unpinned" at the format level: no real .ptau/.r1cs is in the reference).  The oracle's
ptau of known toxic waste (tau, alpha, beta) is built from Lagrange evaluations at every level,
independently of the known-tau setup that gives the expected key (gamma = delta = 1).

CPU: the two oracle paths agree where they overlap (the H section is the ptau's odd level-(k+1)
Lagrange points; alpha1/beta1/beta2 are its first points), and a proof made with the new key
verifies under it.
GPU: zkp_zkey_new(r1cs, ptau) is byte-identical to the oracle's key -- including section 10's
circuit hash (csHash, oracle/mpc.py; recalled snarkjs composition, parity unpinned) -- and the GPU
prover's proofs with it verify."""
import json
import os
import struct

import pytest

from oracle import binfile, bn254, circuit, groth16, mpc, setup
import zkp_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
TAU, ALPHA, BETA = 0x1234567890ABCDEF1122334455667788 % groth16.R, 987654321987654321, 555555555555
_cache = {}


def _case(name):
    if name not in _cache:
        m = json.load(open(os.path.join(GOLD, "manifest.json")))["circuits"][name]
        r1cs, w = circuit.gen_circuit(m["n_vars"], m["n_constraints"], m["n_public"], m["circuit_seed"])
        n = circuit.domain_size_for(r1cs.n_constraints, r1cs.n_public)
        k = n.bit_length() - 1
        ptau = setup.ptau_known_tau(k + 1, TAU, ALPHA, BETA)
        z = setup.zkey_new(r1cs, TAU, ALPHA, BETA)
        # section 10 of a new key: the circuit hash (oracle/mpc.py) and no contributions
        z.extra["mpc"] = {"cs_hash": mpc.cs_hash(z, TAU), "contributions": []}
        _cache[name] = (r1cs, w, n, k, ptau, z)
    return _cache[name]


def _sections(buf, magic):
    _, secs = binfile.read_binfile(buf, magic, 1)
    return {sid: buf[v[0][0]:v[0][0] + v[0][1]] for sid, v in secs.items()}


def test_oracle_ptau_and_new_key_agree():
    r1cs, w, n, k, ptau, z = _case("tiny")
    ps = _sections(ptau, b"ptau")
    power = struct.unpack_from("<I", ps[1], 36)[0]
    assert power == k + 1 and len(ps[12]) == ((2 << power) - 1) * 64 and len(ps[13]) == ((2 << power) - 1) * 128
    lvl = (2 << k) - 1  # level k + 1 starts at point 2^(k+1) - 1
    odd = b"".join(ps[12][(lvl + 2 * j + 1) * 64:(lvl + 2 * j + 2) * 64] for j in range(n))
    assert odd == b"".join(bn254.g1_to_lem(p) for p in z.h)
    assert ps[4][:64] == bn254.g1_to_lem(z.alpha1) and ps[5][:64] == bn254.g1_to_lem(z.beta1)
    assert ps[6] == bn254.g2_to_lem(z.beta2)
    assert z.gamma2 == bn254.G2_GEN and z.delta2 == bn254.G2_GEN and z.delta1 == bn254.G1_GEN
    proof, pub = groth16.prove(z, w, 11, 13)
    assert groth16.verify_with_zkey(z, pub, proof)
    rs = _sections(binfile.write_r1cs(r1cs), b"r1cs")
    assert struct.unpack_from("<IIII", rs[1], 36) == (r1cs.n_vars, 0, r1cs.n_public, r1cs.n_vars - 1 - r1cs.n_public)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny", "small"])
def test_gpu_zkey_new_matches_oracle_and_proves(name):
    r1cs, w, n, k, ptau, z = _case(name)
    out = zkp_amd.zkey_new(binfile.write_r1cs(r1cs), ptau)
    want = binfile.write_zkey(z)
    assert len(out) == len(want)
    if out != want:  # name the first differing section
        got, exp = _sections(out, b"zkey"), _sections(want, b"zkey")
        assert [s for s in exp if got.get(s) != exp[s]] == []
    (a, b, c), pub = zkp_amd.Prover(out).prove_raw(binfile.write_wtns(w))
    assert groth16.verify_with_zkey(z, pub, {"A": a, "B": b, "C": c})


@pytest.mark.gpu
def test_gpu_zkey_new_errors():
    r1cs, w, n, k, ptau, z = _case("tiny")
    small = setup.ptau_known_tau(k, TAU, ALPHA, BETA)  # power k: no level k + 1 for H
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.zkey_new(binfile.write_r1cs(r1cs), small)
    assert e.value.status == 1 and "too big" in e.value.message
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.zkey_new(b"xxxx" + binfile.write_r1cs(r1cs)[4:], ptau)
    assert e.value.status == 3
