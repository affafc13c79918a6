#!/usr/bin/env python3
"""Time the phase-2 contribution math (zkp_zkey_contribute: delta -> k*delta, sections
2, 8, 9) on the Venmo-shaped synthetic zkey on one MI355X.  Reference: `snarkjs zkey
contribute` is part of the 782 s / 3 h key generation (zkp-mooc-hackathon-submission.md:98-99)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))
import zkp_amd  # noqa: E402
from zkp_amd import synth  # noqa: E402

circ = synth.Circuit.venmo(0x5A4B5032)
zk = circ.zkey(0x5A4B5033)  # library-owned buffer, passed without copying
t0 = time.time()
out = zkp_amd.zkey_contribute(zk, 0x1234567890ABCDEF)
dt = time.time() - t0
assert len(out) == zk.len
n_l = circ.n_vars - circ.n_public - 1
print(json.dumps({"op": "zkey_contribute (delta -> k*delta)", "zkey_bytes": zk.len, "seconds": round(dt, 3),
                  "points_scaled": n_l + circ.domain_size + 2,
                  "note": "includes host<->device copies of sections 8 and 9 (PCIe)"}))
