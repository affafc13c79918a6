#!/usr/bin/env python3
"""Isolated witness-plan build timing (zkp_bench_plan, compacted plan, c = 18) on the Venmo-shaped
synthetic witness (bool_pct 70 and 0): the hand-written LDS-staged sort with the tiled pass C
(default) against ZKP_W_SORT=rocprim (onesweep + hipcub scan + a host round trip); and the H plan
(2^23 uniform scalars, c = 20, dense) with the one-workgroup-per-sub-bin pass C (default) against
ZKP_HS_TILED_C=1.  usage: wplan_bench.py [iters=10]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))
import zkp_amd  # noqa: E402
from zkp_amd import synth  # noqa: E402


def wtns_scalars(w: bytes) -> bytes:
    # .wtns v2: 12-byte file header, section 1 (12 + 4 + 32 + 4 bytes), section 2 header (12)
    return w[12 + 12 + 40 + 12:]


def timed(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: v for k, v in env.items() if v is not None})
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
    try:
        return round(fn(), 4)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main(iters=10):
    out = {}
    for pct in (70, 0):
        circ = synth.Circuit.venmo(0x5A4B5032, bool_pct=pct)
        sc = wtns_scalars(circ.witness(1))
        assert len(sc) == 32 * circ.n_vars
        for name, env in (("hsort", {"ZKP_W_SORT": None}), ("rocprim", {"ZKP_W_SORT": "rocprim"})):
            out["witness_bool%d_%s_ms" % (pct, name)] = timed(
                env, lambda: zkp_amd.bench_plan(sc, 18, False, 2, iters))
    rng = np.random.default_rng(0x5A4B5032)
    w = rng.integers(0, 2 ** 32, size=(1 << 23, 8), dtype=np.uint64).astype(np.uint32)
    w[:, 7] &= 0x1FFFFFFF
    h = w.tobytes()
    for name, env in (("fine", {"ZKP_HS_TILED_C": None}), ("tiled", {"ZKP_HS_TILED_C": "1"})):
        out["h_plan_c20_%s_ms" % name] = timed(env, lambda: zkp_amd.bench_plan(h, 20, True, 2, iters))
    print(json.dumps(out))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
