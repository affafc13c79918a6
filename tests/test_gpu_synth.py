"""The C++/HIP synthetic zkey generator (tooling for benchmarks) must produce the
exact bytes of the Python oracle's setup for the same seeds."""
import os

import pytest

from oracle import binfile, circuit, setup
from zkp_amd import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(12, 10, 2, 11, 12), (200, 230, 26, 21, 22)])
def test_synth_zkey_bytes_match_oracle(shape):
    nv, nc, npub, cseed, sseed = shape
    c = synth.Circuit(nv, nc, npub, cseed)
    got = c.zkey(sseed).bytes()
    r1cs, _ = circuit.gen_circuit(nv, nc, npub, cseed)
    want = binfile.write_zkey(setup.setup(r1cs, sseed))
    assert got == want


def test_synth_points_match_oracle():
    from oracle import bn254
    sc = synth.scalars(3, 0, 64)
    ks = [int.from_bytes(sc[32 * i:32 * i + 32], "little") for i in range(64)]
    g1 = synth.points(sc)
    g2 = synth.points(sc, g2=True)
    for i in (0, 1, 63):
        assert bn254.g1_from_lem(g1[64 * i:64 * i + 64]) == bn254.g1_mul(bn254.G1_GEN, ks[i])
        assert bn254.g2_from_lem(g2[128 * i:128 * i + 128]) == bn254.g2_mul(bn254.G2_GEN, ks[i])
