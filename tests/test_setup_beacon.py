"""§8f row 4 (setup acceleration): `snarkjs zkey beacon <in> <out> $BEACON 10` (reference
dizkus-scripts/3_gen_chunk_zkey.sh:36).

The beacon's secret comes from snarkjs@0.4.22 / ffjavascript (absent from the reference):
chained SHA-256, a ChaCha20 word stream, Fr.fromRng.  oracle/beacon.py restates it; its
ChaCha block function and block counter are pinned by OpenSSL's chacha20 keystream
(tests/golden/beacon_vectors.json, made by tests/golden/make_beacon_vectors.py), SHA-256 by
hashlib; the composition has no snarkjs fixture (parity unpinned).
CPU: the oracle against the OpenSSL vectors; the C ABI's host-only derivation
(zkp_beacon_secret) against the oracle.
GPU: zkp_zkey_beacon == the oracle's contribution with the beacon's secret, byte for byte, with
the contribution record (oracle/mpc.py) appended to section 10."""
import json
import os

import pytest

from oracle import beacon, binfile, groth16, mpc, setup
import zkp_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
VEC = json.load(open(os.path.join(GOLD, "beacon_vectors.json")))


def test_oracle_chacha_matches_openssl():
    for c in VEC["chacha20_openssl"]:
        r = beacon.ChaCha(c["seed"])
        words = [r.next_u32() for _ in range(len(c["keystream_hex"]) // 8)]
        assert b"".join(w.to_bytes(4, "little") for w in words).hex() == c["keystream_hex"]


def test_oracle_beacon_regression_vectors():
    for b in VEC["beacon_oracle"]:
        raw = bytes.fromhex(b["beacon_hex"])
        assert beacon.beacon_hash(raw, b["num_iterations_exp"]).hex() == b["hash_hex"]
        assert beacon.beacon_secret(raw, b["num_iterations_exp"]) == int(b["k"])


@pytest.mark.parametrize("raw,e", [(bytes(range(1, 33)), 10), (b"\x00", 0), (b"", 3), (bytes(range(200)), 2),
                                   (b"\xff" * 55, 1), (b"\xab" * 56, 1), (b"\xcd" * 64, 0)])
def test_capi_beacon_secret_matches_oracle(raw, e):
    """Host-only C ABI call (no GPU): SHA-256 padding edges (55/56/64-byte messages, empty)."""
    assert zkp_amd.beacon_secret(raw, e) == beacon.beacon_secret(raw, e)


def test_capi_beacon_rejects_huge_exponent():
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.beacon_secret(b"\x01", 64)
    assert e.value.status == 1


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny", "small"])
def test_gpu_zkey_beacon_matches_oracle_and_proves(name):
    zk = open(os.path.join(GOLD, "circuit_%s.zkey" % name), "rb").read()
    wt = open(os.path.join(GOLD, "circuit_%s.wtns" % name), "rb").read()
    raw = bytes.fromhex(VEC["beacon_oracle"][0]["beacon_hex"])
    out = zkp_amd.zkey_beacon(zk, raw, 10, name="Final Beacon phase2")
    z2, k = mpc.beacon(binfile.read_zkey(zk), raw, 10, name="Final Beacon phase2")
    assert k == beacon.beacon_secret(raw, 10)
    assert z2.delta1 == setup.contribute_delta(binfile.read_zkey(zk), k).delta1
    assert out == binfile.write_zkey(z2)  # including the type-1 record appended to section 10
    (a, b, c), pub = zkp_amd.Prover(out).prove_raw(wt)
    assert groth16.verify_with_zkey(z2, pub, {"A": a, "B": b, "C": c})
