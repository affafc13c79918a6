"""§8f row 4 at size: the setup chain `zkey new` -> `zkey contribute -e` ->
`zkey beacon 10` (reference dizkus-scripts/3_gen_chunk_zkey.sh:18,27,36) on a 2^16-domain
synthetic circuit, and the GPU-built inputs of tools/bench_setup.py (the Venmo-shape timing) pinned
to the oracle at a small size.

* The synthetic circuit's .r1cs (zkp_synth_r1cs) equals the oracle's write_r1cs of the same
  generator, and the known-tau .ptau built on the GPU (zkp_synth_ptau) equals the oracle's
  ptau_known_tau of the same tau, alpha, beta (setup.toxic_from_seed), byte for byte.
* At 2^16: zkey new's point sections equal the known-tau key with gamma = delta = 1 (a different
  computation: QAP evaluation at tau + fixed-base products), the contributed and beaconed key proves,
  the proof at fixed r, s equals oracle/cpu's (independent C++ prover) and passes the host pairing
  verifier.  Format parity of .r1cs / .ptau / the MPC records stays unpinned (recalled layouts)."""
import struct

import pytest

from oracle import binfile, circuit, setup
import zkp_amd
from zkp_amd import synth

pytestmark = pytest.mark.gpu
SEED_C, SEED_S = 0x5A4B5032, 0x5A4B5033
BEACON = bytes.fromhex("0102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f20")


def _sections(buf):
    n = struct.unpack_from("<I", buf, 8)[0]
    o, out = 12, {}
    for _ in range(n):
        sid, ln = struct.unpack_from("<IQ", buf, o)
        out[sid] = buf[o + 12:o + 12 + ln]
        o += 12 + ln
    return out


def test_synth_r1cs_and_ptau_equal_oracle():
    nv, nc, npub = 40, 48, 3
    r1cs, _ = circuit.gen_circuit(nv, nc, npub, SEED_C)
    assert synth.Circuit(nv, nc, npub, SEED_C).r1cs().bytes() == binfile.write_r1cs(r1cs)
    tw = setup.toxic_from_seed(SEED_S)
    want = setup.ptau_known_tau(4, tw["tau"], tw["alpha"], tw["beta"])
    assert synth.ptau(4, SEED_S).bytes() == want


def test_setup_chain_2_16_proves_like_oracle_cpu():
    from oracle import cpu_oracle
    circ = synth.Circuit(60000, 65000, 26, SEED_C)
    k = circ.domain_size.bit_length() - 1
    assert circ.domain_size == 1 << 16
    z0 = zkp_amd.zkey_new(circ.r1cs(), synth.ptau(k + 1, SEED_S))
    ref = circ.zkey(SEED_S, unit_gamma_delta=True).bytes()
    a, b = _sections(z0), _sections(ref)
    assert [s for s in range(2, 10) if a[s] != b[s]] == []
    z1 = zkp_amd.zkey_contribute_entropy(z0, "scale test", rand64=bytes(range(64)), name="first contribution")
    z2 = zkp_amd.zkey_beacon(z1, BEACON, 10, name="Final Beacon phase2")
    assert len(z2) > len(z0)
    wit = circ.witness(77)
    p = zkp_amd.Prover(z2)
    proof, pub = p.prove_raw(wit, 0x1234567, 0x7654321)
    p.close()
    cpu, _ = cpu_oracle.prove(z2, wit, 0x1234567, 0x7654321, threads=8)
    assert cpu == proof
    assert zkp_amd.proof_verify(z2, proof, pub)
