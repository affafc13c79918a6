#!/usr/bin/env python3
"""Phase-2 setup at the Venmo shape on one MI355X:
`snarkjs zkey new` -> `zkey contribute -e` -> `zkey beacon <hex> 10` (reference
dizkus-scripts/3_gen_chunk_zkey.sh:18,27,36; published cost 782 s for the key and 3 h chunked,
zkp-mooc-hackathon-submission.md:98-99), timed end to end through the C ABI, then a proof with the
final key.

Inputs (tooling, not timed as setup): the synthetic Venmo-shaped circuit as a circom .r1cs and a
prepared known-tau .ptau of power lg(domain) + 1 built on the GPU (zkp_synth_ptau).  Checks:
  * zkey new's sections 2..9 byte-identical to the known-tau key of the same tau, alpha, beta with
    gamma = delta = 1 (zkp_synth_zkey_ex: direct QAP evaluation + fixed-base products, a different
    computation from zkey new's ptau-point linear combinations);
  * the proof with the final key at fixed r, s equals oracle/cpu's proof (independent C++ prover) and
    passes the host pairing verifier (zkp_proof_verify).
usage: bench_setup.py [--scale 1.0] [--out profiles/bench_setup_venmo_r04.json]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))
import zkp_amd  # noqa: E402
from zkp_amd import synth  # noqa: E402

CIRCUIT_SEED, SETUP_SEED = 0x5A4B5032, 0x5A4B5033
BEACON = bytes.fromhex("0102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f20")
RAND64 = bytes(range(7, 71))
R_FIX, S_FIX = 0x1234567, 0x7654321


def sections(buf: bytes):
    import struct
    n = struct.unpack_from("<I", buf, 8)[0]
    o, out = 12, {}
    for _ in range(n):
        sid, ln = struct.unpack_from("<IQ", buf, o)
        out[sid] = (o + 12, ln)
        o += 12 + ln
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the Venmo shape")
    ap.add_argument("--out", default="")
    ap.add_argument("--cpu-check", action="store_true", help="prove with oracle/cpu too (about 15 s on 16 cores)")
    args = ap.parse_args()
    v = synth.VENMO
    circ = synth.Circuit(int(v["n_vars"] * args.scale), int(v["n_constraints"] * args.scale), v["n_public"],
                         CIRCUIT_SEED)
    k = circ.domain_size.bit_length() - 1
    t0 = time.time()
    r1cs = circ.r1cs()
    t_r1cs = time.time() - t0
    t0 = time.time()
    ptau = synth.ptau(k + 1, SETUP_SEED, device=0)
    t_ptau = time.time() - t0
    print("# r1cs %.2f GB %.1f s, ptau power %d %.2f GB %.1f s" % (r1cs.len / 1e9, t_r1cs, k + 1, ptau.len / 1e9,
                                                                    t_ptau), file=sys.stderr, flush=True)
    res = {"op": "zkey new -> zkey contribute -e -> zkey beacon 10, then a proof",
           "circuit": {"n_vars": circ.n_vars, "n_constraints": circ.n_constraints, "n_public": circ.n_public,
                       "domain": circ.domain_size},
           "inputs": {"r1cs_bytes": r1cs.len, "ptau_power": k + 1, "ptau_bytes": ptau.len,
                      "ptau_synth_s": round(t_ptau, 2), "note": "known-tau tooling inputs, not timed as setup"}}
    t0 = time.time()
    z0 = zkp_amd.zkey_new(r1cs, ptau)
    res["zkey_new_s"] = round(time.time() - t0, 3)
    del ptau
    ref = circ.zkey(SETUP_SEED, device=0, unit_gamma_delta=True).bytes()
    sa, sb = sections(z0), sections(ref)
    same = {}
    for sid in range(2, 10):
        (oa, la), (ob, lb) = sa[sid], sb[sid]
        same[str(sid)] = la == lb and z0[oa:oa + la] == ref[ob:ob + lb]
    res["zkey_new_vs_known_tau_sections_equal"] = same
    del ref
    t0 = time.time()
    z1 = zkp_amd.zkey_contribute_entropy(z0, "venmo-shape contribution", rand64=RAND64, name="first contribution")
    res["zkey_contribute_s"] = round(time.time() - t0, 3)
    t0 = time.time()
    z2 = zkp_amd.zkey_beacon(z1, BEACON, 10, name="Final Beacon phase2")
    res["zkey_beacon_s"] = round(time.time() - t0, 3)
    res["total_s"] = round(res["zkey_new_s"] + res["zkey_contribute_s"] + res["zkey_beacon_s"], 3)
    res["zkey_bytes"] = len(z2)
    del z0, z1
    wit = circ.witness(4242)
    p = zkp_amd.Prover(z2, devices=[0])
    (a, b, c), pub = p.prove_raw(wit, R_FIX, S_FIX)
    p.close()
    res["final_key_proof_verifies"] = zkp_amd.proof_verify(z2, (a, b, c), pub)
    if args.cpu_check:
        from oracle import cpu_oracle
        t0 = time.time()
        cpu, _ = cpu_oracle.prove(z2, wit, R_FIX, S_FIX)
        res["final_key_proof_equals_oracle_cpu"] = cpu == (a, b, c)
        res["oracle_cpu_s"] = round(time.time() - t0, 1)
    res["published"] = {"zkey_generation_s": 782, "chunked_zkey_s": 10800,
                        "source": "zkp-mooc-hackathon-submission.md:98-99 (snarkjs on CPU, other hardware)"}
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
