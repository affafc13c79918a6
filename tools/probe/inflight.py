#!/usr/bin/env python3
"""Probe: throughput with 1 vs 2 proofs in flight on one GPU (two Prover instances, each with
its own resident key and streams, fed from two host threads).  Venmo-shaped synthetic
circuit as in bench.py.  usage: inflight.py [proofs]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))
import zkp_amd  # noqa: E402
from zkp_amd import synth  # noqa: E402
import bench  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 16
circ = synth.Circuit.venmo(bench.CIRCUIT_SEED)
wit = bench.gen_witnesses(circ, [1, 2, 3, 4])
zk = circ.zkey(bench.SETUP_SEED, device=0, threads=16)
R, S = 0x1234567, 0x7654321
provers = []
for k in range(2):
    p = zkp_amd.Prover(zk, devices=[0])
    for i, w in enumerate(wit):
        p.stage(w, slot=i)
    provers.append(p)
ref = provers[0].prove_staged_raw(0, R, S)
assert provers[1].prove_staged_raw(0, R, S) == ref
for p in provers:
    for i in range(2):
        p.prove_staged_raw(i, R, S)


def run(p, n, off):
    for i in range(n):
        p.prove_staged_raw((i + off) % 4, R, S)


for rep in range(2):
    t0 = time.perf_counter()
    run(provers[0], K, 0)
    t1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(provers[k], K // 2, k)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    t2 = time.perf_counter() - t0
    print("inflight1 %.3f ms/proof  inflight2 %.3f ms/proof  gain %.1f%%" % (t1 / K * 1e3, t2 / K * 1e3,
          (t1 / t2 - 1) * 100), flush=True)
