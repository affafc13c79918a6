"""GPU parity at the shapes of BASELINE.json configs[3] and configs[4], through the C ABI,
against the C++ CPU restatement of the oracle (oracle/cpu) -- VERDICT r2 "next" item 1.

* configs[3] (batch of Venmo-circuit proofs): a Venmo-shaped zkp_prove_batch from HOST
  memory with two pipelines per GPU (ZKP_INFLIGHT=2, the bench default): 32 proofs over 8
  distinct witnesses.  Every proof equals the staged proof of the same witness, two equal
  oracle/cpu's proof, and one verifies.
* configs[4] (one 2^24-constraint proof split by point range): the S24 circuit of bench.py
  (2^24 - 27 constraints, nPublic 26) proved unsplit on one GPU and as 8 balanced slices
  with the distributed quotient (ZKP_SPLIT_BALANCE=1, parts 0..2 extend one quotient vector
  each, every part joins its own domain slice), emulated on device 0 as bench.py --mode split
  does in one process (the slice exchange is a device copy here; RCCL carries it on a
  multi-GPU node).  Both combined proofs equal oracle/cpu's proof at fixed r, s and verify.
  This runs the c = 21 / 22 dense H plans of 2^21-2^22 slices, the balanced ranges at G = 8
  and the 2^24 coset NTT against an independent implementation.
"""
import os
import sys

import pytest

from oracle import binfile, cpu_oracle, groth16
import zkp_amd
from zkp_amd import synth

pytestmark = pytest.mark.gpu

CIRCUIT_SEED, SETUP_SEED = 0x5A4B5032, 0x5A4B5033  # bench.py's
R_FIX, S_FIX = 0x1234567, 0x7654321
S24 = dict(n_vars=16_000_000, n_constraints=(1 << 24) - 27, n_public=26)  # bench.py S24 (configs[4])


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 8
    return max(1, min(16, n))  # the GPU box's CPU share is 16


def _say(msg):
    print("[test_gpu_configs] " + msg, file=sys.stderr, flush=True)


def _zkey_view(zk):
    import ctypes
    return memoryview((ctypes.c_uint8 * zk.len).from_address(ctypes.cast(zk.ptr, ctypes.c_void_p).value))


def _verify(zk, pub, proof):
    vk = binfile.read_zkey_vk(_zkey_view(zk))
    (a, b, c) = proof
    return groth16.verify(vk["ic"], vk["alpha1"], vk["beta2"], vk["gamma2"], vk["delta2"], pub,
                          {"A": a, "B": b, "C": c})


def _cpu_proof(zk, wit):
    cpu, _ = cpu_oracle.prove(None, wit, R_FIX, S_FIX, threads=_threads(), zkey_ptr=zk.ptr, zkey_len=zk.len)
    return cpu


@pytest.mark.timeout(600)
def test_venmo_batch_inflight_from_host(monkeypatch):
    monkeypatch.setenv("ZKP_INFLIGHT", "2")
    circ = synth.Circuit.venmo(CIRCUIT_SEED, bool_pct=70)
    wits = [circ.witness(700 + i) for i in range(8)]
    zk = circ.zkey(SETUP_SEED, device=0, threads=_threads())
    _say("venmo circuit, 8 witnesses, zkey ready")
    p = zkp_amd.Prover(zk, devices=[0])
    try:
        staged = []
        for i, w in enumerate(wits):
            p.stage(w, slot=i)
            staged.append(p.prove_staged_raw(i, R_FIX, S_FIX))
        order = [(3 * j + j // 8) % 8 for j in range(32)]  # each witness 4 times, interleaved
        batch = p.prove_batch_raw([wits[i] for i in order], [R_FIX] * 32, [S_FIX] * 32)
    finally:
        p.close()
    _say("staged + 32-proof batch done")
    assert len(batch) == 32
    for j, i in enumerate(order):
        assert batch[j] == staged[i], (j, i)
    assert len({s[0] for s in staged}) == 8  # distinct witnesses -> distinct proofs
    for i in (0, 5):
        assert staged[i][0] == _cpu_proof(zk, wits[i]), i
    _say("two proofs equal oracle/cpu")
    assert _verify(zk, staged[5][1], staged[5][0])


@pytest.mark.timeout(900)
def test_s24_split_8_balanced_distq_vs_cpu(monkeypatch):
    import torch
    from zkp_amd.dist import split_range
    monkeypatch.setenv("ZKP_SPLIT_BALANCE", "1")
    circ = synth.Circuit(S24["n_vars"], S24["n_constraints"], S24["n_public"], CIRCUIT_SEED)
    assert circ.domain_size == 1 << 24
    wit = circ.witness(1)
    zk = circ.zkey(SETUP_SEED, device=0, threads=_threads())
    _say("S24 circuit, witness, zkey (%.2f GB) ready" % (zk.len / 1e9))
    G = 8
    provers = [zkp_amd.Prover(zk, devices=[0], part=k, nparts=G) for k in range(G)]
    try:
        n = provers[0].domain_size
        full = [torch.empty(n * 32, dtype=torch.uint8, device="cuda:0") for _ in range(3)]
        for k, pr in enumerate(provers):
            pr.stage(wit, 0)
            mine = [v for v in range(3) if v % G == k]
            if mine:
                pr.quotient_part_staged(0, sum(1 << v for v in mine),
                                        [full[v].data_ptr() if v in mine else None for v in range(3)])
        parts = []
        for k, pr in enumerate(provers):
            lo, hi = split_range(n, k, G)
            assert (lo, hi) == split_range(n, k, G, balance=True)
            sl = [full[v][lo * 32:hi * 32].clone() for v in range(3)]
            torch.cuda.synchronize(0)
            parts.append(pr.prove_partial_ext_staged(0, [t.data_ptr() for t in sl]))
        del full, sl
    finally:
        for pr in provers:
            pr.close()
    split_proof, pub = zkp_amd.proof_combine_raw(zk, parts, wit, R_FIX, S_FIX)
    _say("8-slice split proof done")
    p = zkp_amd.Prover(zk, devices=[0])
    try:
        unsplit, pub2 = p.prove_raw(wit, R_FIX, S_FIX)
    finally:
        p.close()
    _say("unsplit proof done")
    assert unsplit == split_proof and pub2 == pub
    assert unsplit == _cpu_proof(zk, wit)
    _say("equal to oracle/cpu")
    assert _verify(zk, pub, unsplit)
