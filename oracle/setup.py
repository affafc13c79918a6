"""INSECURE known-tau Groth16 setup producing snarkjs-layout zkeys — TEST INFRASTRUCTURE ONLY.

Restates what ``snarkjs groth16 setup`` + contributions produce (reference call
sites ``dizkus-scripts/3_gen_chunk_zkey.sh:18-36``), with the
toxic waste derived from a seed so that zkeys can be made offline:

* A_i, B_i, C_i = sum_c M[c][i] * L_c(tau) over the domain w = Fr.w[log2 n],
  including the nPublic+1 "input" rows A[nConstraints+i][i] = 1.
* sec5 A_i*G1, sec6 B_i*G1, sec7 B_i*G2,
  sec3 IC_i = (beta A_i + alpha B_i + C_i)/gamma * G1   (i <= nPublic),
  sec8 C_i  = (beta A_i + alpha B_i + C_i)/delta * G1   (i >  nPublic),
  sec9 H_j  = delta^-1 * L^(2n)_(2j+1)(tau) * G1      (odd Lagrange points of the 2n domain).
"""
from __future__ import annotations

from . import bn254
from .binfile import ZKey
from .circuit import R1CS, SplitMix64, domain_size_for
from .ntt import ROOTS, coset_gen, log2_exact

R = bn254.R


def toxic_from_seed(seed: int):
    rng = SplitMix64(seed, 7)
    vals = []
    for _ in range(5):
        v = 0
        while v == 0:
            v = rng.fr()
        vals.append(v)
    tau, alpha, beta, gamma, delta = vals
    return dict(tau=tau, alpha=alpha, beta=beta, gamma=gamma, delta=delta)


def _batch_inv(xs):
    pref = []
    acc = 1
    for x in xs:
        pref.append(acc)
        acc = acc * x % R
    ai = bn254.inv(acc, R)
    out = [0] * len(xs)
    for i in range(len(xs) - 1, -1, -1):
        out[i] = ai * pref[i] % R
        ai = ai * xs[i] % R
    return out


def lagrange_at(tau: int, n: int, w: int):
    """L_c(tau) = (tau^n - 1)/n * w^c / (tau - w^c) for c < n."""
    pw = []
    cur = 1
    for _ in range(n):
        pw.append(cur)
        cur = cur * w % R
    dens = [(tau - x) % R for x in pw]
    if any(d == 0 for d in dens):
        raise ValueError("tau in domain")
    invs = _batch_inv(dens)
    z = (pow(tau, n, R) - 1) * bn254.inv(n, R) % R
    return [z * pw[c] % R * invs[c] % R for c in range(n)]


def h_scalars(tau: int, n: int):
    """L^(2n)_(2j+1)(tau) for j < n  (coset points g w^j, g = Fr.w[log2 n + 1])."""
    g = coset_gen(n)
    w = ROOTS[log2_exact(n)]
    pts = []
    cur = g
    for _ in range(n):
        pts.append(cur)
        cur = cur * w % R
    invs = _batch_inv([(tau - x) % R for x in pts])
    z = (pow(tau, 2 * n, R) - 1) * bn254.inv(2 * n, R) % R
    return [z * pts[j] % R * invs[j] % R for j in range(n)]


def qap_at_tau(r1cs: R1CS, tau: int, n: int):
    L = lagrange_at(tau, n, ROOTS[log2_exact(n)])
    nv = r1cs.n_vars
    A = [0] * nv
    B = [0] * nv
    C = [0] * nv
    for c, (a, b, cc) in enumerate(r1cs.constraints):
        lc = L[c]
        for s, v in a:
            A[s] = (A[s] + v * lc) % R
        for s, v in b:
            B[s] = (B[s] + v * lc) % R
        for s, v in cc:
            C[s] = (C[s] + v * lc) % R
    for i in range(r1cs.n_public + 1):
        A[i] = (A[i] + L[r1cs.n_constraints + i]) % R
    return A, B, C


def zkey_coefs(r1cs: R1CS):
    """Section-4 coefficient list (matrix, constraint, signal, plain value)."""
    out = []
    for c, (a, b, _) in enumerate(r1cs.constraints):
        for s, v in a:
            out.append((0, c, s, v))
        for s, v in b:
            out.append((1, c, s, v))
    for i in range(r1cs.n_public + 1):
        out.append((0, r1cs.n_constraints + i, i, 1))
    return out


def setup(r1cs: R1CS, seed: int) -> ZKey:
    return setup_toxic(r1cs, toxic_from_seed(seed))


def setup_toxic(r1cs: R1CS, tw: dict) -> ZKey:
    tau, alpha, beta, gamma, delta = tw["tau"], tw["alpha"], tw["beta"], tw["gamma"], tw["delta"]
    n = domain_size_for(r1cs.n_constraints, r1cs.n_public)
    A, B, C = qap_at_tau(r1cs, tau, n)
    g1 = bn254.FixedBase(bn254.G1_GEN)
    g2 = bn254.FixedBase(bn254.G2_GEN, g2=True)
    ginv = bn254.inv(gamma, R)
    dinv = bn254.inv(delta, R)
    npub = r1cs.n_public
    lin = [(beta * A[i] + alpha * B[i] + C[i]) % R for i in range(r1cs.n_vars)]
    ic = bn254.batch_to_affine_g1([g1.mul_jac(lin[i] * ginv) for i in range(npub + 1)])
    cpts = bn254.batch_to_affine_g1([g1.mul_jac(lin[i] * dinv) for i in range(npub + 1, r1cs.n_vars)])
    apts = bn254.batch_to_affine_g1([g1.mul_jac(x) for x in A])
    b1pts = bn254.batch_to_affine_g1([g1.mul_jac(x) for x in B])
    b2pts = [g2.mul(x) for x in B]
    hs = h_scalars(tau, n)
    hpts = bn254.batch_to_affine_g1([g1.mul_jac(x * dinv) for x in hs])
    z = ZKey(
        n_vars=r1cs.n_vars, n_public=npub, domain_size=n,
        alpha1=g1.mul(alpha), beta1=g1.mul(beta), beta2=g2.mul(beta), gamma2=g2.mul(gamma),
        delta1=g1.mul(delta), delta2=g2.mul(delta),
        ic=ic, coefs=zkey_coefs(r1cs), a=apts, b1=b1pts, b2=b2pts, c=cpts, h=hpts,
    )
    z.extra["toxic"] = tw
    return z


def vkey_json(z: ZKey) -> dict:
    """snarkjs ``zkey export verificationkey`` layout (reference app/src/helpers/vkey.ts:1-219)."""
    def g1o(p):
        return [str(p[0]), str(p[1]), "1"]

    def g2o(p):
        return [[str(p[0][0]), str(p[0][1])], [str(p[1][0]), str(p[1][1])], ["1", "0"]]

    return {
        "protocol": "groth16",
        "curve": "bn128",
        "nPublic": z.n_public,
        "vk_alpha_1": g1o(z.alpha1),
        "vk_beta_2": g2o(z.beta2),
        "vk_gamma_2": g2o(z.gamma2),
        "vk_delta_2": g2o(z.delta2),
        "vk_alphabeta_12": bn254.f12_to_obj(bn254.pairing_snarkjs(z.alpha1, z.beta2)),
        "IC": [g1o(p) for p in z.ic],
    }


def contribute_delta(z: ZKey, k: int) -> ZKey:
    """Group arithmetic of a phase-2 contribution with secret k (snarkjs `zkey contribute`
    / `zkey beacon`, reference dizkus-scripts/3_gen_chunk_zkey.sh:27,36): delta -> k*delta,
    so delta1, delta2 are multiplied by k and the L (C) and H sections, which carry
    delta^-1, by k^-1.  The contribution transcript (section 10) is not modelled."""
    import copy
    k %= bn254.R
    if k == 0:
        raise ValueError("contribution scalar must be nonzero mod r")
    ki = bn254.inv(k, bn254.R)
    out = copy.copy(z)
    out.delta1 = bn254.g1_mul(z.delta1, k)
    out.delta2 = bn254.g2_mul(z.delta2, k)
    out.c = [None if p is None else bn254.g1_mul(p, ki) for p in z.c]
    out.h = [None if p is None else bn254.g1_mul(p, ki) for p in z.h]
    return out


# ------------------------------------------------------------------ `zkey new` from a ptau


def zkey_new(r1cs: R1CS, tau: int, alpha: int, beta: int) -> ZKey:
    """What ``snarkjs zkey new <r1cs> <ptau>`` produces (reference dizkus-scripts/
    3_gen_chunk_zkey.sh:18) from a ptau of toxic waste (tau, alpha, beta): the phase-2 key
    before any contribution, gamma = delta = 1 (the generators).  Equal to the known-tau setup
    with those values, which is how the GPU builder (zkp_zkey_new) is checked."""
    return setup_toxic(r1cs, dict(tau=tau, alpha=alpha, beta=beta, gamma=1, delta=1))


def ptau_known_tau(power: int, tau: int, alpha: int, beta: int) -> bytes:
    """An INSECURE ptau of known toxic waste (tau, alpha, beta), binfile.write_ptau layout."""
    from .binfile import write_ptau
    g1 = bn254.FixedBase(bn254.G1_GEN)
    g2 = bn254.FixedBase(bn254.G2_GEN, g2=True)
    N = 1 << power
    pw = [1]
    for _ in range(2 * N - 2):
        pw.append(pw[-1] * tau % R)
    tau_g1 = bn254.batch_to_affine_g1([g1.mul_jac(x) for x in pw])
    tau_g2 = [g2.mul(x) for x in pw[:N]]
    alpha_tau = bn254.batch_to_affine_g1([g1.mul_jac(alpha * x % R) for x in pw[:N]])
    beta_tau = bn254.batch_to_affine_g1([g1.mul_jac(beta * x % R) for x in pw[:N]])
    lag = []
    for p in range(power + 1):
        lag += lagrange_at(tau, 1 << p, ROOTS[p])
    l_tau_g1 = bn254.batch_to_affine_g1([g1.mul_jac(x) for x in lag])
    l_tau_g2 = [g2.mul(x) for x in lag]
    l_alpha = bn254.batch_to_affine_g1([g1.mul_jac(alpha * x % R) for x in lag])
    l_beta = bn254.batch_to_affine_g1([g1.mul_jac(beta * x % R) for x in lag])
    return write_ptau(power, tau_g1, tau_g2, alpha_tau, beta_tau, g2.mul(beta), l_tau_g1, l_tau_g2, l_alpha,
                      l_beta)
