#!/usr/bin/env python3
"""Summarise tools/gpu/ab.sh outputs: proofs/s, ms per proof and the H-launch frac per run, base vs new.
usage: ab_summary.py <tag>   (reads gpurun_out/<tag>/ab_*.json)"""
import glob
import json
import statistics
import sys

tag = sys.argv[1]
arms = {"base": [], "new": []}
for f in sorted(glob.glob("gpurun_out/%s/ab_*.json" % tag)):
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no bench line")
        continue
    d = json.loads(lines[-1])
    arm = "base" if "/ab_base_" in f else "new"
    arms[arm].append(d["value"])
    print("%-36s %.4f proofs/s  %.3f ms  H frac %.4f" % (f, d["value"], d["ms_per_step"], d["roofline"]["frac"]))
for arm, v in arms.items():
    if v:
        print("%s: median %.4f proofs/s over %d runs" % (arm, statistics.median(v), len(v)))
