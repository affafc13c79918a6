#!/usr/bin/env python3
"""Probe: batch throughput with one vs two proof pipelines on the same GPU
(Prover(devices=[0]) vs Prover(devices=[0, 0]); witnesses from host memory)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))
import zkp_amd
from zkp_amd import synth
circ = synth.Circuit.venmo(0x5A4B5032)
wit = [circ.witness(i + 1) for i in range(8)]
zk = circ.zkey(0x5A4B5033)
for devs in ([0], [0, 0]):
    p = zkp_amd.Prover(zk, devices=devs)
    p.prove_batch_raw(wit[:len(devs) * 2], [3] * (len(devs) * 2), [5] * (len(devs) * 2))
    t0 = time.time()
    p.prove_batch_raw(wit * 2, [3] * 16, [5] * 16)
    dt = time.time() - t0
    print("devices=%s: 16 proofs in %.3f s -> %.2f proofs/s" % (devs, dt, 16 / dt), flush=True)
    p.close()
    del p
