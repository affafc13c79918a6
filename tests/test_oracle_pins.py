"""Pin the CPU oracle to what the reference itself holds:
curve constants, the G2 generator and coordinate orders, the vkey points, the
snarkjs GT value vk_alphabeta_12, the Solidity verifying key, the public-signal
layout and the stale proof fixture.  Data comes from tests/golden/reference_fixtures.json
(extracted by tests/golden/extract_reference_fixtures.py)."""
import json
import os

import pytest

from oracle import bn254, groth16

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_fixtures.json")))
VK = FIX["vkey_ts"]
SOL = FIX["verifier_sol"]


def g1(o):
    return (int(o[0]), int(o[1]))


def g2_vkey(o):  # vkey.ts order [[x.c0, x.c1], [y.c0, y.c1]]
    return ((int(o[0][0]), int(o[0][1])), (int(o[1][0]), int(o[1][1])))


def g2_sol(v):  # Verifier.sol order [x.c1, x.c0], [y.c1, y.c0]
    v = [int(x) for x in v]
    return ((v[1], v[0]), (v[3], v[2]))


def test_field_constants_match_verifier_sol():
    assert int(SOL["q"]) == bn254.P            # Verifier.sol:52
    assert int(SOL["snark_scalar_field"]) == bn254.R  # Verifier.sol:341


def test_g2_generator_and_solidity_coordinate_order():
    gen = g2_sol(SOL["g2_generator_sol_order"])
    assert gen == bn254.G2_GEN and bn254.g2_on_curve(gen)
    v = [int(x) for x in SOL["g2_generator_sol_order"]]
    assert not bn254.g2_on_curve(((v[0], v[1]), (v[2], v[3])))  # the raw Solidity order is [c1, c0]


def test_vkey_points_on_curve():
    assert bn254.g1_on_curve(g1(VK["vk_alpha_1"]))
    for k in ("vk_beta_2", "vk_gamma_2", "vk_delta_2"):
        assert bn254.g2_on_curve(g2_vkey(VK[k]))
    assert len(VK["IC"]) == VK["nPublic"] + 1 == 27
    for p in VK["IC"]:
        assert bn254.g1_on_curve(g1(p))


def test_pairing_reproduces_vk_alphabeta_12():
    """snarkjs' e(alpha1, beta2) (vkey.ts:52-82) — pins Fq12 tower, Miller loop and final exp."""
    got = bn254.pairing_snarkjs(g1(VK["vk_alpha_1"]), g2_vkey(VK["vk_beta_2"]))
    assert bn254.f12_to_obj(got) == VK["vk_alphabeta_12"]


def test_solidity_vk_matches_vkey_except_delta():
    assert g1(SOL["alfa1"]) == g1(VK["vk_alpha_1"])
    assert g2_sol(SOL["beta2_sol_order"]) == g2_vkey(VK["vk_beta_2"])
    assert g2_sol(SOL["gamma2_sol_order"]) == g2_vkey(VK["vk_gamma_2"])
    assert [g1(p) for p in SOL["IC"]] == [g1(p) for p in VK["IC"]]
    d = g2_sol(SOL["delta2_sol_order"])
    assert bn254.g2_on_curve(d) and d != g2_vkey(VK["vk_delta_2"])


def _ramp_proof():
    rp = FIX["ramp_test_proof"]
    h = lambda x: int(x, 16)
    A = (h(rp["a"][0]), h(rp["a"][1]))
    B = ((h(rp["b"][0][1]), h(rp["b"][0][0])), (h(rp["b"][1][1]), h(rp["b"][1][0])))  # calldata is [c1, c0]
    C = (h(rp["c"][0]), h(rp["c"][1]))
    return {"A": A, "B": B, "C": C}, [h(x) for x in rp["signals"]]


def test_ramp_fixture_layout():
    proof, sig = _ramp_proof()
    assert bn254.g1_on_curve(proof["A"]) and bn254.g1_on_curve(proof["C"]) and bn254.g2_on_curve(proof["B"])
    # the same calldata shape our exporter produces (reference SubmitOrderOnRampForm.tsx:36-46)
    a, b, c, _ = groth16.solidity_calldata(proof, sig)
    rp = FIX["ramp_test_proof"]
    assert [int(x, 16) for x in b[0]] == [int(x, 16) for x in rp["b"][0]]
    # Ramp.sol:266-292 signal order vs circuit/input.json
    inp = FIX["input_json"]
    assert sig[7:24] == [int(x) for x in inp["modulus"]]
    assert sig[24] == int(inp["order_id"]) and sig[25] == int(inp["claim_id"])
    assert len(sig) == VK["nPublic"]


def test_ramp_fixture_does_not_verify_under_either_vkey():
    """Documented in SURVEY.md §0.3: the stale fixture pins layouts, not verification."""
    proof, sig = _ramp_proof()
    ic = [g1(p) for p in VK["IC"]]
    alpha, beta, gamma = g1(VK["vk_alpha_1"]), g2_vkey(VK["vk_beta_2"]), g2_vkey(VK["vk_gamma_2"])
    for delta in (g2_vkey(VK["vk_delta_2"]), g2_sol(SOL["delta2_sol_order"])):
        assert groth16.verify(ic, alpha, beta, gamma, delta, sig, proof) is False
