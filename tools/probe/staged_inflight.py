#!/usr/bin/env python3
"""Probe: staged proofs with 1 vs T host threads on ONE prover (ZKP_INFLIGHT = T pipelines per
device sharing the base tables; concurrent zkp_prove_staged callers take the idle pipelines).
Every proof is checked against the single-flight proof of the same witness.
usage: staged_inflight.py [proofs] [threads]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))
K = int(sys.argv[1]) if len(sys.argv) > 1 else 16
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2
os.environ.setdefault("ZKP_INFLIGHT", str(T))
import zkp_amd  # noqa: E402
from zkp_amd import synth  # noqa: E402
import bench  # noqa: E402

circ = synth.Circuit.venmo(bench.CIRCUIT_SEED)
wit = bench.gen_witnesses(circ, [1, 2, 3, 4])
zk = circ.zkey(bench.SETUP_SEED, device=0, threads=16)
R, S = 0x1234567, 0x7654321
p = zkp_amd.Prover(zk, devices=[0])
for i, w in enumerate(wit):
    p.stage(w, slot=i)
refs = [p.prove_staged_raw(i, R, S) for i in range(4)]
bad = []


def run(n, off):
    for i in range(n):
        s = (i + off) % 4
        if p.prove_staged_raw(s, R, S) != refs[s]:
            bad.append(s)


run(4, 0)
for rep in range(2):
    t0 = time.perf_counter()
    run(K, 0)
    t1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(K // T, k)) for k in range(T)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    t2 = time.perf_counter() - t0
    print("hwq %s threads %d: 1 thread %.3f ms/proof, %d threads %.3f ms/proof, gain %.1f%%, mismatches %d"
          % (os.environ.get("GPU_MAX_HW_QUEUES", "default"), T, t1 / K * 1e3, T, t2 / (K // T * T) * 1e3,
             (t1 / K / (t2 / (K // T * T)) - 1) * 100, len(bad)), flush=True)
