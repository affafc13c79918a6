#!/usr/bin/env python3
"""Coset extension of 1 vector vs the batched extension of 3 (every pass one launch over A, B, C,
as the prover runs them): ms per vector at 2^20 and 2^23, best of 3 x 20, rounds alternating.
usage: ntt_batch.py [rounds=2] -> one JSON line per (round, log_n)"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "zk-p2p-onramp_amd"))
import zkp_amd  # noqa: E402

for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    for k in (20, 23):
        one = min(zkp_amd.bench_ntt(k, warmup=3, iters=20) for _ in range(3))
        three = min(zkp_amd.bench_ntt(k, warmup=3, iters=20, count=3) for _ in range(3))
        print(json.dumps({"round": rnd, "log_n": k, "ms_one_vector": round(one, 4), "ms_three_batched": round(three, 4),
                          "ms_per_vector_batched": round(three / 3, 4), "gain": round(one / (three / 3), 3)}), flush=True)
