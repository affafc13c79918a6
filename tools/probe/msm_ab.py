#!/usr/bin/env python3
"""G1 MSM 2^20 accumulate timing per library (ZKP_LIB_PATH per child), libraries alternated R rounds.
usage: msm_ab.py R lib1 [lib2 ...]"""
import json, os, subprocess, sys

CHILD = r'''
import json, sys
sys.path.insert(0, "zk-p2p-onramp_amd")
import zkp_amd
from zkp_amd import synth
n = 1 << 20
pts = synth.points(synth.scalars(7, 0, n), g2=False, device=0)
sc = synth.scalars(7, 1, n)
best = None
for _ in range(3):
    st, _r = zkp_amd.bench_msm(pts, sc, g2=False, warmup=2, iters=10, device=0)
    if best is None or st["ms_accumulate"] < best["ms_accumulate"]:
        best = st
best["lib"] = sys.argv[1]
print(json.dumps(best))
'''

def main():
    rounds, libs = int(sys.argv[1]), sys.argv[2:]
    for _ in range(rounds):
        for lib in libs:
            env = dict(os.environ, ZKP_LIB_PATH=os.path.abspath(lib))
            out = subprocess.run([sys.executable, "-c", CHILD, lib], env=env, capture_output=True, text=True,
                                 timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            print(line[0] if line else json.dumps({"lib": lib, "rc": out.returncode, "err": out.stderr[-400:]}),
                  flush=True)

if __name__ == "__main__":
    main()
