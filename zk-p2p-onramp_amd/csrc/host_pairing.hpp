// Host-side BN254 optimal-ate pairing for the optional verify-before-return of a proof
// (SURVEY.md §5 failure detection; the reference verifies every proof right after proving:
// dizkus-scripts/5_gen_proof.sh:14-21, `snarkjs groth16 verify`, whose equation is restated from
// contracts/Verifier.sol:340-358).  Not on the throughput path: a check costs a few ms of one host
// core, off by default.
//
// Tower: Fq2 = Fq[u]/(u^2 + 1), Fq6 = Fq2[v]/(v^3 - xi), Fq12 = Fq6[w]/(w^2 - v), xi = 9 + u
// (SURVEY.md Appendix C).  Miller loop over 6u + 2 with affine steps (the slopes' inversions of all
// pairs of a multi-pairing shared by Montgomery's trick), the two Frobenius correction lines, then
// ffjavascript's final exponentiation: the easy part (p^6 - 1)(p^2 + 1) and the Fuentes-Castaneda
// hard part, so a single pairing equals the GT value snarkjs reports (e.g. vk_alphabeta_12 of
// reference app/src/helpers/vkey.ts:52-82, which pins it: tests/test_host_pairing.py).
#pragma once
#include "host_ec.hpp"

namespace zkp {
namespace host {

struct Fq6 {
  Fq2 c0, c1, c2;
};
struct Fq12 {
  Fq6 c0, c1;  // c0 + c1 w
};

Fq12 fq12_one();
Fq12 fq12_mul(const Fq12& a, const Fq12& b);
bool fq12_is_one(const Fq12& a);
// product of the Miller loops of n pairs (pairs with a point at infinity contribute 1)
Fq12 miller_loop_multi(const Affine<Fq>* ps, const Affine<Fq2>* qs, int n);
Fq12 final_exponentiation(const Fq12& f);
// snarkjs-convention GT element e(P, Q)
Fq12 pairing(const Affine<Fq>& p, const Affine<Fq2>& q);

bool g1_on_curve(const Affine<Fq>& p);  // y^2 = x^3 + 3 (infinity: true)
bool g2_on_curve(const Affine<Fq2>& p);  // y^2 = x^3 + 3/(9+u)
// r * Q == infinity (G2 subgroup membership; the twist's cofactor is not 1)
bool g2_in_subgroup(const Affine<Fq2>& p);

// Groth16 verification (Verifier.sol:340-358 restated): vk_x = IC[0] + sum_i in_i IC[i+1];
// e(-A, B) e(alpha1, beta2) e(vk_x, gamma2) e(C, delta2) == 1.  ic: n_public + 1 points; pub:
// n_public standard-form scalars (each must be < r, as Verifier.sol:347 requires).
struct VerifyingKey {
  Affine<Fq> alpha1;
  Affine<Fq2> beta2, gamma2, delta2;
  const Affine<Fq>* ic = nullptr;
  int n_public = 0;
};
bool groth16_verify(const VerifyingKey& vk, const U256* pub, const Affine<Fq>& a, const Affine<Fq2>& b,
                    const Affine<Fq>& c);

}  // namespace host
}  // namespace zkp
