#!/usr/bin/env python3
"""Summarise tools/gpu/ab.sh / abenv.sh outputs: proofs/s, ms per proof and the H-launch frac per run, per arm
(ab.sh: base vs new; abenv.sh: one arm per ZKP_MSM setting).
usage: ab_summary.py <tag>   (reads gpurun_out/<tag>/ab_<arm>_<round>.json)"""
import collections
import glob
import json
import re
import statistics
import sys

tag = sys.argv[1]
arms = collections.OrderedDict()
for f in sorted(glob.glob("gpurun_out/%s/ab_*.json" % tag)):
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no bench line")
        continue
    d = json.loads(lines[-1])
    arm = re.match(r".*/ab_(.*)_\d+\.json$", f).group(1)
    arms.setdefault(arm, []).append(d["value"])
    print("%-36s %.4f proofs/s  %.3f ms  H frac %.4f" % (f, d["value"], d["ms_per_step"], d["roofline"]["frac"]))
for arm, v in arms.items():
    if v:
        print("%s: median %.4f proofs/s over %d runs" % (arm, statistics.median(v), len(v)))
