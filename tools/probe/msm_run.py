#!/usr/bin/env python3
"""One short configs[1] G1 MSM 2^20 bench for rocprofv3 (kernel trace / counter passes)."""
import json, sys
sys.path.insert(0, "zk-p2p-onramp_amd")
import zkp_amd
from zkp_amd import synth
n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
pts = synth.points(synth.scalars(7, 0, n), g2=False, device=0)
sc = synth.scalars(7, 1, n)
st, _ = zkp_amd.bench_msm(pts, sc, g2=False, warmup=2, iters=5, device=0)
print(json.dumps(st))
