"""Groth16 prove/verify restatement — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

``prove`` restates snarkjs 0.4.22 ``groth16_prove`` (upstream pin reference
``package-lock.json:3884-3896``; call sites ``dizkus-scripts/5_gen_proof.sh:8``,
``circuit/scripts/generate_proof_groth16.sh:11``, ``app/src/helpers/zkp.ts:94``)
step by step as SURVEY.md §8a rows A1–A10 describe it, with the blinding scalars
r, s injectable (snarkjs draws them from ``Fr.random()``).

``verify`` restates ``contracts/Verifier.sol:340-358``:
    vk_x = IC[0] + sum input[i] * IC[i+1]   (every input < r, ``:347``)
    e(-A, B) e(alpha1, beta2) e(vk_x, gamma2) e(C, delta2) == 1
"""
from __future__ import annotations

import json

from . import bn254, ntt
from .binfile import ZKey

R = bn254.R


class ProveError(Exception):
    pass


def build_abc(z: ZKey, w):
    """A4 buildABC1: A_T[c] += v*w[s] (matrix 0), B_T likewise, C_T = A_T * B_T."""
    n = z.domain_size
    A = [0] * n
    B = [0] * n
    for m, c, s, v in z.coefs:
        if m == 0:
            A[c] = (A[c] + v * w[s]) % R
        else:
            B[c] = (B[c] + v * w[s]) % R
    C = [A[i] * B[i] % R for i in range(n)]
    return A, B, C


def quotient_scalars(z: ZKey, w):
    """A4-A8: the H-MSM scalars P_j = A(g w^j) B(g w^j) - C(g w^j) (standard form)."""
    n = z.domain_size
    A, B, C = build_abc(z, w)
    g = ntt.coset_gen(n)
    odd = []
    for X in (A, B, C):
        coeffs = ntt.ifft(X)
        odd.append(ntt.fft(ntt.batch_apply_key(coeffs, 1, g)))
    Ao, Bo, Co = odd
    return [(Ao[j] * Bo[j] - Co[j]) % R for j in range(n)]


def msm_g1(points, scalars):
    acc = bn254.G1J_INF
    for p, k in zip(points, scalars):
        if p is not None and k % R:
            acc = bn254.g1j_add(acc, bn254.g1j_from_affine(bn254.g1_mul(p, k)))
    return bn254.g1j_to_affine(acc)


def msm_g2(points, scalars):
    acc = bn254.G2J_INF
    for p, k in zip(points, scalars):
        if p is not None and k % R:
            acc = bn254.g2j_add(acc, bn254.g2j_from_affine(bn254.g2_mul(p, k)))
    return bn254.g2j_to_affine(acc)


def prove(z: ZKey, w, r: int, s: int):
    """Returns (proof dict of ints, public signals).  proof = {'A': g1, 'B': g2, 'C': g1}."""
    if len(w) != z.n_vars:
        raise ProveError("Invalid witness length")
    w = [x % R for x in w]
    h = quotient_scalars(z, w)
    pa = msm_g1(z.a, w)
    pb1 = msm_g1(z.b1, w)
    pb = msm_g2(z.b2, w)
    pc = msm_g1(z.c, w[z.n_public + 1:])
    ph = msm_g1(z.h, h)
    A = bn254.g1_add(bn254.g1_add(pa, z.alpha1), bn254.g1_mul(z.delta1, r))
    B = bn254.g2_add(bn254.g2_add(pb, z.beta2), bn254.g2_mul(z.delta2, s))
    B1 = bn254.g1_add(bn254.g1_add(pb1, z.beta1), bn254.g1_mul(z.delta1, s))
    C = bn254.g1_add(pc, ph)
    C = bn254.g1_add(C, bn254.g1_mul(A, s))
    C = bn254.g1_add(C, bn254.g1_mul(B1, r))
    C = bn254.g1_add(C, bn254.g1_mul(z.delta1, (-r * s) % R))
    return {"A": A, "B": B, "C": C}, w[1:z.n_public + 1]


def split_range(n: int, part: int, nparts: int, balance: bool = False):
    """[lo, hi) of slice `part` of n items in nparts contiguous ranges (as prover.hip split_range);
    balance (ZKP_SPLIT_BALANCE=1 there): for nparts > 3, parts 0..2 (the quotient-vector owners)
    weigh max(1, 11 - nparts) and the others 11."""
    if not balance or nparts <= 3:
        return n * part // nparts, n * (part + 1) // nparts
    wq = max(1, 11 - nparts)  # see prover.hip split_range
    cum = lambda k: wq * min(k, 3) + 11 * max(k - 3, 0)  # noqa: E731
    return n * cum(part) // cum(nparts), n * cum(part + 1) // cum(nparts)


def partial_sums(z: ZKey, w, part: int, nparts: int, h=None, balance: bool = False):
    """MSM partial sums of point slice `part` of `nparts` (the point-range split of one proof,
    SURVEY.md §8e E1(2)): witness-indexed sections A, B1, B2, C over [wlo, whi) (C's base of
    signal i is z.c[i - nPublic - 1]), H over [hlo, hhi) of the domain.  Summing the partials
    of all parts gives prove()'s pa, pb1, pb, pc, ph."""
    w = [x % R for x in w]
    if h is None:
        h = quotient_scalars(z, w)
    wlo, whi = split_range(z.n_vars, part, nparts, balance)
    hlo, hhi = split_range(z.domain_size, part, nparts, balance)
    c0 = z.n_public + 1
    cidx = [i for i in range(max(wlo, c0), whi)]
    return {
        "a": msm_g1(z.a[wlo:whi], w[wlo:whi]),
        "b1": msm_g1(z.b1[wlo:whi], w[wlo:whi]),
        "c": msm_g1([z.c[i - c0] for i in cidx], [w[i] for i in cidx]),
        "h": msm_g1(z.h[hlo:hhi], h[hlo:hhi]),
        "b2": msm_g2(z.b2[wlo:whi], w[wlo:whi]),
    }


def verify(vk_ic, alpha1, beta2, gamma2, delta2, public, proof) -> bool:
    if len(public) + 1 != len(vk_ic):
        raise ValueError("verifier-bad-input")
    vk_x = None
    for i, x in enumerate(public):
        if x >= R:
            raise ValueError("verifier-gte-snark-scalar-field")
        vk_x = bn254.g1_add(vk_x, bn254.g1_mul(vk_ic[i + 1], x))
    vk_x = bn254.g1_add(vk_x, vk_ic[0])
    return bn254.pairing_prod_is_one([
        (bn254.g1_neg(proof["A"]), proof["B"]),
        (alpha1, beta2),
        (vk_x, gamma2),
        (proof["C"], delta2),
    ])


def verify_with_zkey(z: ZKey, public, proof) -> bool:
    return verify(z.ic, z.alpha1, z.beta2, z.gamma2, z.delta2, public, proof)


# ------------------------------------------------------------------ JSON (snarkjs formatting)


def proof_to_json_obj(proof) -> dict:
    A, B, C = proof["A"], proof["B"], proof["C"]
    return {
        "pi_a": [str(A[0]), str(A[1]), "1"],
        "pi_b": [[str(B[0][0]), str(B[0][1])], [str(B[1][0]), str(B[1][1])], ["1", "0"]],
        "pi_c": [str(C[0]), str(C[1]), "1"],
        "protocol": "groth16",
        "curve": "bn128",
    }


def js_stringify(obj) -> str:
    """JSON.stringify(obj, null, 1)."""
    return json.dumps(obj, indent=1)


def proof_from_json_obj(o) -> dict:
    A = (int(o["pi_a"][0]), int(o["pi_a"][1]))
    B = ((int(o["pi_b"][0][0]), int(o["pi_b"][0][1])), (int(o["pi_b"][1][0]), int(o["pi_b"][1][1])))
    C = (int(o["pi_c"][0]), int(o["pi_c"][1]))
    return {"A": A, "B": B, "C": C}


def verify_calldata(z: ZKey, calldata: str) -> bool:
    """On-chain acceptance of `zkey export soliditycalldata` text: restates
    Verifier.sol:359-375 verifyProof(a, b, c, input) -> verify(:340-358).  b arrives in the
    EIP-197 [c1, c0] order (Pairing.G2Point stores X as [c1, c0], Verifier.sol:184-188)."""
    a, b, c, inputs = json.loads("[" + calldata + "]")
    h = lambda x: int(x, 16)
    A = (h(a[0]), h(a[1]))
    B = ((h(b[0][1]), h(b[0][0])), (h(b[1][1]), h(b[1][0])))
    C = (h(c[0]), h(c[1]))
    try:
        return verify_with_zkey(z, [h(x) for x in inputs], {"A": A, "B": B, "C": C})
    except ValueError:  # require() failures revert
        return False


def solidity_calldata(proof, public):
    """``zkey export soliditycalldata`` shape: G2 pairs reversed to [c1, c0]
    (reference SubmitOrderOnRampForm.tsx:36-46, Verifier.sol:366-369)."""
    A, B, C = proof["A"], proof["B"], proof["C"]
    a = [hex(A[0]), hex(A[1])]
    b = [[hex(B[0][1]), hex(B[0][0])], [hex(B[1][1]), hex(B[1][0])]]
    c = [hex(C[0]), hex(C[1])]
    return a, b, c, [hex(x) for x in public]
