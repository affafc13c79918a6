#!/usr/bin/env python3
"""Generate the committed golden fixtures from the CPU oracle (oracle/).

Run from the repo root:  python3 tests/golden/make_golden.py
Outputs (all small; deterministic from the seeds below):
  circuit_<name>.zkey / .wtns        snarkjs-layout proving key + witness
  proof_<name>.json / public_<name>.json   oracle proof at fixed r, s (JSON.stringify(x,null,1))
  vkey_<name>.json                   `zkey export verificationkey` layout
  quotient_<name>.bin                H-MSM scalars P_j (32-byte LE, domain entries)
  msm_g1_<n>.bin / msm_g2_<n>.bin    points (zkey layout) | scalars | expected affine result
  ntt_<k>.json                       input, forward, inverse, coset-extend vectors
  manifest.json                      parameters + sha256 of every file
The reference holds no prover fixture that verifies, so these are
oracle-generated; tests/test_oracle_*.py pin the oracle itself to the reference's
own constants and vkey (vk_alphabeta_12).
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import binfile, bn254, circuit, groth16, ntt, setup  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
R = bn254.R

CIRCUITS = {
    # name: (n_vars, n_constraints, n_public, circuit_seed, setup_seed, r, s)
    "tiny": (12, 10, 2, 11, 12, 0x1234, 0x5678),
    "small": (200, 230, 26, 21, 22, 7 ** 60 % R, 11 ** 70 % R),
    "venmo_mini": (1000, 1034, 26, 31, 32, 3 ** 150 % R, 5 ** 120 % R),
}


def write(name, data):
    mode = "w" if isinstance(data, str) else "wb"
    with open(os.path.join(OUT, name), mode) as f:
        f.write(data)


def gen_circuit(name, params):
    nv, nc, npub, cseed, sseed, r, s = params
    r1cs, w = circuit.gen_circuit(nv, nc, npub, cseed)
    assert circuit.check_witness(r1cs, w)
    z = setup.setup(r1cs, sseed)
    zbytes = binfile.write_zkey(z)
    write("circuit_%s.zkey" % name, zbytes)
    write("circuit_%s.wtns" % name, binfile.write_wtns(w))
    z = binfile.read_zkey(zbytes)
    proof, pub = groth16.prove(z, w, r, s)
    assert groth16.verify_with_zkey(z, pub, proof)
    write("proof_%s.json" % name, groth16.js_stringify(groth16.proof_to_json_obj(proof)))
    write("public_%s.json" % name, groth16.js_stringify([str(x) for x in pub]))
    write("vkey_%s.json" % name, json.dumps(setup.vkey_json(z), indent=1))
    q = groth16.quotient_scalars(z, w)
    write("quotient_%s.bin" % name, b"".join(bn254.int_to_le(x) for x in q))
    return {"n_vars": nv, "n_constraints": nc, "n_public": npub, "domain": z.domain_size,
            "circuit_seed": cseed, "setup_seed": sseed, "r": str(r), "s": str(s)}


def msm_vectors_g1(n, seed):
    rng = circuit.SplitMix64(seed, 0)
    g = bn254.FixedBase(bn254.G1_GEN)
    pts = []
    for i in range(n):
        pts.append(g.mul(rng.fr() or 1))
    # edge cases: infinity, duplicate, negation pair
    pts[3] = None
    pts[5] = pts[4]
    pts[7] = bn254.g1_neg(pts[6])
    scal = [rng.fr() for _ in range(n)]
    scal[0] = 0
    scal[1] = 1
    scal[2] = R - 1
    scal[5] = scal[4]          # P + P with equal digits -> doubling inside a bucket
    scal[7] = scal[6]          # P + (-P) in the same bucket -> infinity
    for i in range(8, min(n, 8 + n // 4)):
        scal[i] = rng.next() & 1  # bit-heavy tail like a circuit witness
    res = groth16.msm_g1(pts, scal)
    blob = b"".join(bn254.g1_to_lem(p) for p in pts) + b"".join(bn254.int_to_le(x) for x in scal)
    blob += bn254.int_to_le(res[0]) + bn254.int_to_le(res[1]) if res else bytes(64)
    return blob


def msm_vectors_g2(n, seed):
    rng = circuit.SplitMix64(seed, 0)
    g = bn254.FixedBase(bn254.G2_GEN, g2=True)
    pts = [g.mul(rng.fr() or 1) for _ in range(n)]
    pts[3] = None
    pts[5] = pts[4]
    pts[7] = bn254.g2_neg(pts[6])
    scal = [rng.fr() for _ in range(n)]
    scal[0] = 0
    scal[1] = 1
    scal[2] = R - 1
    scal[5] = scal[4]
    scal[7] = scal[6]
    res = groth16.msm_g2(pts, scal)
    blob = b"".join(bn254.g2_to_lem(p) for p in pts) + b"".join(bn254.int_to_le(x) for x in scal)
    if res:
        blob += b"".join(bn254.int_to_le(v) for v in (res[0][0], res[0][1], res[1][0], res[1][1]))
    else:
        blob += bytes(128)
    return blob


def ntt_vectors(k, seed):
    rng = circuit.SplitMix64(seed, 2)
    n = 1 << k
    a = [rng.fr() for _ in range(n)]
    fwd = ntt.fft(a)
    inv = ntt.ifft(a)
    g = ntt.coset_gen(n)
    cos = ntt.fft(ntt.batch_apply_key(ntt.ifft(a), 1, g))
    return json.dumps({"k": k, "input": [str(x) for x in a], "forward": [str(x) for x in fwd],
                       "inverse": [str(x) for x in inv], "coset": [str(x) for x in cos]})


def main():
    manifest = {"circuits": {}, "msm": {}, "ntt": {}}
    for name, params in CIRCUITS.items():
        print("circuit", name, flush=True)
        manifest["circuits"][name] = gen_circuit(name, params)
    for n, seed in ((64, 0x5A4B5032), (1024, 0x5A4B5033)):
        print("msm g1", n, flush=True)
        write("msm_g1_%d.bin" % n, msm_vectors_g1(n, seed))
        manifest["msm"]["g1_%d" % n] = {"n": n, "seed": seed}
    for n, seed in ((64, 0x5A4B5034), (256, 0x5A4B5035)):
        print("msm g2", n, flush=True)
        write("msm_g2_%d.bin" % n, msm_vectors_g2(n, seed))
        manifest["msm"]["g2_%d" % n] = {"n": n, "seed": seed}
    for k in (1, 4, 10, 12):
        write("ntt_%d.json" % k, ntt_vectors(k, 0x5A4B5032 + k))
        manifest["ntt"]["k%d" % k] = {"k": k}
    files = sorted(f for f in os.listdir(OUT) if f not in ("manifest.json", "make_golden.py") and not f.startswith("."))
    manifest["sha256"] = {f: hashlib.sha256(open(os.path.join(OUT, f), "rb").read()).hexdigest() for f in files}
    write("manifest.json", json.dumps(manifest, indent=1, sort_keys=True))
    print("wrote", len(files), "files")


if __name__ == "__main__":
    main()
