#!/usr/bin/env python3
"""Isolated MSM plan-build timing (zkp_bench_plan): the Venmo H plan (2^23 uniform scalars,
c = 20, dense) grouped by the hand-written LDS-staged bucket sort vs rocprim onesweep, and the
compacted witness plan for reference.  usage: plan_bench.py [log_n=23] [iters=10] [only_hsort=0]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "zk-p2p-onramp_amd"))
import zkp_amd  # noqa: E402


def main(lg=23, iters=10, only_hsort=0):
    n = 1 << lg
    rng = np.random.default_rng(0x5A4B5032)
    w = rng.integers(0, 2 ** 32, size=(n, 8), dtype=np.uint64).astype(np.uint32)
    w[:, 7] &= 0x1FFFFFFF  # < 2^253 < r: uniform-like Fr values
    sc = w.tobytes()
    c = lg - 3
    out = {"n": n, "c": c}
    os.environ.pop("ZKP_H_SORT", None)
    out["dense_hsort_ms"] = zkp_amd.bench_plan(sc, c, True, 2, iters)
    if only_hsort:
        print(json.dumps(out))
        return
    os.environ["ZKP_H_SORT"] = "rocprim"
    out["dense_rocprim_ms"] = zkp_amd.bench_plan(sc, c, True, 2, iters)
    os.environ.pop("ZKP_H_SORT", None)
    out["compacted_rocprim_ms"] = zkp_amd.bench_plan(sc, c, False, 2, iters)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
