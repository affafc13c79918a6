#!/usr/bin/env python3
"""Witness-plan (or H-plan, --which h) window bits under different witness mixes: for each
bool_pct (percent of bit-valued defining steps of the synthetic Venmo-shaped circuit) build
the circuit, two witnesses and its known-tau key once, then for every witness-plan width c
(ZKP_MSM "w=<c>": the base tables depend on c, so one prover per c) time staged proofs.
Every timed proof is compared with the first c's proof of the same witness.
usage: wsweep.py [--bools 0,70,90] [--cs 17,18,19,20] [--steps 8] -> one JSON line per (bool, c)"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))
import zkp_amd  # noqa: E402
from zkp_amd import synth  # noqa: E402

CIRCUIT_SEED, SETUP_SEED = 0x5A4B5032, 0x5A4B5033
R_FIX, S_FIX = 0x1234567, 0x7654321


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bools", default="0,70,90")
    ap.add_argument("--cs", default="17,18,19,20")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2, help="passes over the widths (alternating order)")
    ap.add_argument("--which", default="w", choices=["w", "h"], help="the witness plan (w) or the H plan (h)")
    args = ap.parse_args()
    for bp in [int(x) for x in args.bools.split(",")]:
        t0 = time.time()
        circ = synth.Circuit.venmo(CIRCUIT_SEED, bool_pct=bp)
        wit = [circ.witness(7001 + i) for i in range(2)]
        zk = circ.zkey(SETUP_SEED, device=0)
        print("# bool_pct %d: circuit, witnesses, key %.1f s" % (bp, time.time() - t0), file=sys.stderr, flush=True)
        ref = None
        cs = [int(x) for x in args.cs.split(",")]
        for rep, c in [(r, c) for r in range(args.reps) for c in (cs if r % 2 == 0 else cs[::-1])]:
            os.environ["ZKP_MSM"] = "%s=%d" % (args.which, c)
            p = zkp_amd.Prover(zk, devices=[0])
            for i, w in enumerate(wit):
                p.stage(w, slot=i)
            first = [p.prove_staged_raw(i, R_FIX, S_FIX) for i in range(2)]
            if ref is None:
                ref = first
            t1 = time.perf_counter()
            res = [p.prove_staged_raw(i % 2, R_FIX, S_FIX) for i in range(args.steps)]
            el = time.perf_counter() - t1
            ok = first == ref and all(r == ref[i % 2] for i, r in enumerate(res))
            print(json.dumps({"bool_pct": bp, args.which: c, "rep": rep, "ms_per_proof": round(el / args.steps * 1e3, 3),
                              "steps": args.steps, "msm": p.msm_config()["witness" if args.which == "w" else "h"], "proofs_equal": ok}), flush=True)
            p.close()
        os.environ.pop("ZKP_MSM", None)
        del zk


if __name__ == "__main__":
    main()
