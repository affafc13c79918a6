#!/usr/bin/env python3
"""configs[1] kernel line A/B: the G1 MSM 2^20 (uniform scalars, fixed-base tables) timed by
zkp_bench_msm in child processes with different ZKP_MSM settings, alternating for R rounds; every
result compared with the first arm's.  usage: msm_ab.py R spec1 [spec2 ...]  ("-" = unset)"""
import json, os, subprocess, sys

CHILD = r'''
import json, sys
sys.path.insert(0, "zk-p2p-onramp_amd")
import zkp_amd
from zkp_amd import synth
n = 1 << 20
pts = synth.points(synth.scalars(0x5A4B5032, 0, n), g2=False)
scal = synth.scalars(0x5A4B5032, 1, n)
best = None
for _ in range(3):
    st, res = zkp_amd.bench_msm(pts, scal, g2=False, warmup=2, iters=10)
    if best is None or st["ms_per_msm"] < best["ms_per_msm"]:
        best = st
print(json.dumps({"ms": best["ms_per_msm"], "acc_ms": best["ms_accumulate"], "res": str(res)}))
'''

def main():
    rounds, specs = int(sys.argv[1]), sys.argv[2:]
    first = None
    for i in range(rounds):
        for spec in specs:
            env = dict(os.environ)
            env.pop("ZKP_MSM", None)
            if spec != "-":
                env["ZKP_MSM"] = spec
            out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            if not line:
                print(json.dumps({"spec": spec, "rc": out.returncode, "err": out.stderr[-400:]}), flush=True)
                continue
            d = json.loads(line[0])
            first = first or d["res"]
            print(json.dumps({"round": i, "spec": spec, "ms": round(d["ms"], 4), "acc_ms": round(d["acc_ms"], 4),
                              "same_result": d["res"] == first}), flush=True)

if __name__ == "__main__":
    main()
