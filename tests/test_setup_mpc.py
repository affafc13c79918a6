"""§8f row 4: the phase-2 ceremony of the reference, end to end, with keys that pass `zkey verify`
(reference dizkus-scripts/3_gen_chunk_zkey.sh:18 `groth16 setup`, :27 `zkey contribute`, :36
`zkey beacon $BEACON 10 -n="Final Beacon phase2"`; the gate circuit/scripts/
generate_keys_phase2_groth16.sh:26 `zkey verify`).

The MPC record (section 10: the circuit hash, the contribution entries) restates snarkjs@0.4.22 /
ffjavascript (oracle/mpc.py, recalled; no snarkjs-written zkey exists offline: the transcript
bytes are parity unpinned).  Pinned here: Blake2b-512 of the C++ code against hashlib.
CPU: the oracle's ceremony verifies under the oracle's `zkey verify`, and every tampering it is
meant to catch is caught (a contribution without its record, a forged record, another circuit).
GPU: new -> contribute -> beacon through the C ABI is byte-identical to the oracle's chain, the
final key passes `zkey verify` against the initial one and proves; the raw primitive
(zkp_zkey_contribute, no record) is rejected."""
import hashlib
import struct
import os

import pytest

from oracle import binfile, bn254, circuit, groth16, mpc, setup
import zkp_amd

TAU, ALPHA, BETA = 0x1234567890ABCDEF1122334455667788 % bn254.R, 987654321987654321, 555555555555
BEACON = bytes.fromhex("0102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f20")
RAND64 = bytes(range(7, 71))
_cache = {}


def _chain(name="tiny"):
    if name not in _cache:
        sizes = {"tiny": (12, 10, 2, 11), "small": (200, 230, 26, 21)}[name]
        r1cs, w = circuit.gen_circuit(*sizes)
        z0 = setup.zkey_new(r1cs, TAU, ALPHA, BETA)
        z0.extra["mpc"] = {"cs_hash": mpc.cs_hash(z0, TAU), "contributions": []}
        z1, _ = mpc.contribute_entropy(z0, RAND64, "some entropy text", name="first contribution")
        z2, _ = mpc.beacon(z1, BEACON, 10, name="Final Beacon phase2")
        _cache[name] = (r1cs, w, z0, z1, z2)
    return _cache[name]


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1000, 65536])
def test_blake2b512_matches_hashlib(n):
    d = bytes((i * 131 + 7) & 255 for i in range(n))
    assert zkp_amd.blake2b512(d) == hashlib.blake2b(d, digest_size=64).digest()


def test_oracle_ceremony_verifies_and_catches_tampering():
    r1cs, w, z0, z1, z2 = _chain()
    init = binfile.write_zkey(z0)
    for z in (z0, z1, z2):
        ok, msg = mpc.zkey_verify(binfile.write_zkey(z), init)
        assert ok, msg
    # the raw group arithmetic without a record (zkp_zkey_contribute): delta no longer matches
    raw = setup.contribute_delta(z2, 5)
    raw.extra = z2.extra
    assert mpc.zkey_verify(binfile.write_zkey(raw), init) == (False, "INVALID: delta1 is not the last deltaAfter")
    # a forged record: deltaAfter claims a delta the proof of knowledge does not support
    import copy
    forged = copy.copy(z2)
    cons = [dict(c) for c in z2.extra["mpc"]["contributions"]]
    cons[-1]["g1_sx"] = bn254.g1_mul(cons[-1]["g1_sx"], 2)
    forged.extra = {"mpc": {"cs_hash": z2.extra["mpc"]["cs_hash"], "contributions": cons}}
    assert not mpc.zkey_verify(binfile.write_zkey(forged), init)[0]
    # the same ceremony on another circuit's initial key
    r1cs_b, _ = circuit.gen_circuit(12, 10, 2, 99)
    other = setup.zkey_new(r1cs_b, TAU, ALPHA, BETA)
    other.extra["mpc"] = {"cs_hash": mpc.cs_hash(other, TAU), "contributions": []}
    assert not mpc.zkey_verify(binfile.write_zkey(z2), binfile.write_zkey(other))[0]
    # proofs with the final key verify
    proof, pub = groth16.prove(z2, w, 3, 5)
    assert groth16.verify_with_zkey(z2, pub, proof)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny", "small"])
def test_gpu_ceremony_matches_oracle_and_verifies(name):
    r1cs, w, z0, z1, z2 = _chain(name)
    n = circuit.domain_size_for(r1cs.n_constraints, r1cs.n_public)
    ptau = setup.ptau_known_tau(n.bit_length(), TAU, ALPHA, BETA)
    k0 = zkp_amd.zkey_new(binfile.write_r1cs(r1cs), ptau)
    assert k0 == binfile.write_zkey(z0)
    k1 = zkp_amd.zkey_contribute_entropy(k0, "some entropy text", rand64=RAND64, name="first contribution")
    assert k1 == binfile.write_zkey(z1)
    k2 = zkp_amd.zkey_beacon(k1, BEACON, 10, name="Final Beacon phase2")
    assert k2 == binfile.write_zkey(z2)
    ok, msg = mpc.zkey_verify(k2, k0)
    assert ok, msg
    (a, b, c), pub = zkp_amd.Prover(k2).prove_raw(binfile.write_wtns(w))
    assert zkp_amd.proof_verify(k2, (a, b, c), pub)
    bad = zkp_amd.zkey_contribute(k2, 12345)  # the primitive: no record -> not a verifiable key
    assert not mpc.zkey_verify(bad, k0)[0]
    fresh = zkp_amd.zkey_contribute_entropy(k1, "other entropy")  # /dev/urandom: a different, valid key
    assert fresh != k2 and mpc.zkey_verify(fresh, k0)[0]


def test_mpc_params_bytes_pinned():
    """The contribution parameter bytes as snarkjs writeMPCParams lays them out: id 1
    (name: length byte, UTF-8), id 2 (numIterationsExp: ONE value byte, no length byte), id 3
    (beacon hash: length byte, bytes); the reader takes id 2's value byte directly."""
    _, _, _, z1, z2 = _chain()
    sec = mpc.write_mpc(z2.extra["mpc"])
    nm = b"Final Beacon phase2"
    want = bytes([1, len(nm)]) + nm + bytes([2, 10, 3, len(BEACON)]) + BEACON
    assert sec.endswith(struct.pack("<I", len(want)) + want)
    back = mpc.read_mpc(sec)["contributions"][-1]
    assert back["numIterationsExp"] == 10 and back["beaconHash"] == BEACON and back["name"] == nm.decode()
    first = mpc.write_mpc(z1.extra["mpc"])
    nm1 = b"first contribution"
    assert first.endswith(struct.pack("<I", 2 + len(nm1)) + bytes([1, len(nm1)]) + nm1)


def test_mpc_name_truncation_utf16_units():
    """snarkjs name.substring(0, 64) counts UTF-16 code units before UTF-8 encoding."""
    assert mpc.mpc_name_bytes("a" * 70) == b"a" * 64
    assert mpc.mpc_name_bytes("é" * 70) == "é".encode() * 64          # 2 UTF-8 bytes, 1 unit
    assert mpc.mpc_name_bytes("\U0001F600" * 40) == "\U0001F600".encode() * 32  # 4 bytes, 2 units
    assert mpc.mpc_name_bytes("a" + "\U0001F600" * 40) == b"a" + "\U0001F600".encode() * 31 + "�".encode()
