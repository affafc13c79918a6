"""The compact witness transfer (prover.hip DevicePipeline::upload + qap.hip k_witness_unpack): the
host sends each block of 64 signals as its 0 / 1 values in the block metadata, its values >= 2^32
(32 B) and the low words of the others; the device expands them.  A proof from a host witness must equal oracle/cpu's proof of the same
witness at the same r, s, whatever the mix of small and large values and wherever they sit in their
block; the witnesses here span several 64K-signal chunks and end in a ragged block.  Witnesses other
than the circuit's own do not satisfy it: the proof is still a deterministic function of (key,
witness, r, s), which is what is compared."""
import numpy as np
import pytest

import zkp_amd
from zkp_amd import synth

pytestmark = pytest.mark.gpu
R_FIX, S_FIX = 0x1234567, 0x7654321
NV = 3 * 65536 + 37  # 3 full chunks + a partial one ending in a ragged block


@pytest.fixture(scope="module")
def setup():
    circ = synth.Circuit(NV, NV + 211, 26, 0x5A4B5032)
    zk = circ.zkey(0x5A4B5033).bytes()
    return circ, zk


def _values(w: bytes, n: int):
    off = len(w) - 32 * n
    return w[:off], np.frombuffer(w, dtype=np.uint32, count=8 * n, offset=off).reshape(n, 8).copy()


def _pattern(kind, v, rng):
    n = v.shape[0]
    if kind == "all_large":
        v[:] = rng.integers(0, 1 << 32, size=v.shape, dtype=np.uint64).astype(np.uint32)
        v[:, 7] &= 0x1FFFFFFF  # < 2^253 < r
    elif kind == "all_small":
        v[:] = 0
        v[:, 0] = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    elif kind == "bits":
        # 0 / 1 values (carried in the block metadata) beside uniform ones, lane by lane at random
        r = rng.integers(0, 1 << 32, size=v.shape, dtype=np.uint64).astype(np.uint32)
        r[:, 7] &= 0x1FFFFFFF
        b = rng.integers(0, 2, size=n, dtype=np.uint32)
        isbit = rng.integers(0, 10, size=n) < 7
        v[:] = r
        v[isbit] = 0
        v[isbit, 0] = b[isbit]
    elif kind == "edges":
        # per lane: 0, 2^32 - 1 (small), 2^32 (large), only the top word set (large), 1, random
        k = np.arange(n) % 6
        v[:] = 0
        v[k == 1, 0] = 0xFFFFFFFF
        v[k == 2, 1] = 1
        v[k == 3, 7] = 0x10000000
        v[k == 4, 0] = 1
        r = rng.integers(0, 1 << 32, size=(int((k == 5).sum()), 8), dtype=np.uint64).astype(np.uint32)
        r[:, 7] &= 0x1FFFFFFF
        v[k == 5] = r
        # whole blocks of one kind next to each other
        v[64 * 5:64 * 6] = 0
        v[64 * 6:64 * 7, 1] = 0xFFFF
    v[0] = 0
    v[0, 0] = 1
    return v


_WANT = {}


def _case(setup, kind):
    """(witness bytes, oracle/cpu proof) of one mix, the proof computed once per module."""
    from oracle import cpu_oracle
    circ, zk = setup
    w = circ.witness(91)
    if kind != "natural":
        head, v = _values(w, circ.n_vars)
        w = head + _pattern(kind, v, np.random.default_rng(5)).tobytes()
    if kind not in _WANT:
        _WANT[kind] = cpu_oracle.prove(zk, w, R_FIX, S_FIX, threads=8)[0]
    return w, _WANT[kind]


@pytest.mark.parametrize("kind", ["natural", "all_large", "all_small", "bits", "edges"])
def test_host_witness_proof_equals_oracle(setup, kind):
    w, want = _case(setup, kind)
    p = zkp_amd.Prover(setup[1], devices=[0])
    try:
        got, _ = p.prove_raw(w, R_FIX, S_FIX)
        p.stage(w, slot=1)
        staged, _ = p.prove_staged_raw(1, R_FIX, S_FIX)
    finally:
        p.close()
    assert got == want
    assert staged == want


def test_host_witness_sequence_on_one_prover(setup):
    """Mixes alternating on one prover: every transfer rewrites the same pinned staging chunks and
    the device must see the new bytes (a stale chunk from the previous witness gives a wrong proof)."""
    seq = ["natural", "all_large", "natural", "edges", "all_large", "bits", "all_small", "all_large"]
    p = zkp_amd.Prover(setup[1], devices=[0])
    try:
        for i, kind in enumerate(seq):
            w, want = _case(setup, kind)
            got, _ = p.prove_raw(w, R_FIX, S_FIX)
            assert got == want, (i, kind)
    finally:
        p.close()


def test_batch_of_mixes_on_inflight_pipelines(setup, monkeypatch):
    """zkp_prove_batch over every mix with two pipelines on the device (ZKP_INFLIGHT=2): transfers of
    different witnesses into different pipelines' staging run concurrently with proofs."""
    monkeypatch.setenv("ZKP_INFLIGHT", "2")
    kinds = ["all_large", "natural", "edges", "bits", "all_small", "natural", "all_large", "edges"]
    cases = [_case(setup, k) for k in kinds]
    p = zkp_amd.Prover(setup[1], devices=[0])
    # these witnesses do not satisfy the circuit (module docstring): the batch's default
    # verify-before-return would refuse their proofs, so it is off here
    p.set_verify(False)
    try:
        got = p.prove_batch_raw([w for w, _ in cases], rs=[R_FIX] * len(cases), ss=[S_FIX] * len(cases))
    finally:
        p.close()
    for i, (g, (_, want)) in enumerate(zip(got, cases)):
        assert g[0] == want, (i, kinds[i])


@pytest.mark.parametrize("kind", ["bits", "all_large"])
@pytest.mark.parametrize("wsel", ["first", "second", "auto"])
def test_witness_configurations_equal_oracle(setup, kind, wsel, monkeypatch):
    """Both resident witness-MSM configurations (window bits c and c + 2, prover.hip pick_wset): a
    proof equals oracle/cpu's whichever one it takes -- forced first or second, or chosen per proof by
    the witness's share of values >= 2^32 (auto: the uniform witness takes the second, the 0/1-heavy
    one the first), from a host witness and from a staged one."""
    monkeypatch.setenv("ZKP_MSM", "wsel=%s" % wsel)
    w, want = _case(setup, kind)
    p = zkp_amd.Prover(setup[1], devices=[0])
    try:
        cfg = p.msm_config()
        assert cfg["witness_second"] and cfg["witness_second"]["c"] == cfg["witness"]["c"] + 2
        got, _ = p.prove_raw(w, R_FIX, S_FIX)
        took = p.timings()["witness_config"]
        p.stage(w, slot=0)
        staged, _ = p.prove_staged_raw(0, R_FIX, S_FIX)
        took_staged = p.timings()["witness_config"]
    finally:
        p.close()
    assert got == want and staged == want
    expect = {"first": 0, "second": 1, "auto": 1 if kind == "all_large" else 0}[wsel]
    assert took == expect and took_staged == expect
