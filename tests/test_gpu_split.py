"""GPU parity of the point-range split of one proof: every
slice's partial sums equal the oracle's bit-exactly, and combining them gives the
golden proof."""
import pytest

import zkp_amd
from test_split import _case, _oracle_partials

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,nparts", [("tiny", 4), ("small", 2), ("small", 3), ("venmo_mini", 5)])
def test_split_partials_bit_exact_and_combine(name, nparts):
    zk, wt, r, s, want = _case(name)
    parts = []
    for k in range(nparts):
        p = zkp_amd.Prover(zk, devices=[0], part=k, nparts=nparts)
        parts.append(p.prove_partial(wt))
        with pytest.raises(zkp_amd.ZkpError):  # a slice cannot make a full proof
            p.prove_raw(wt, r, s)
        p.close()
    assert parts == _oracle_partials(zk, wt, nparts)
    (a, b, c), _ = zkp_amd.proof_combine_raw(zk, parts, wt, r, s)
    assert {"A": a, "B": b, "C": c} == want


def test_full_prover_partial_is_part_0_of_1():
    zk, wt, r, s, want = _case("small")
    p = zkp_amd.Prover(zk)
    part = p.prove_partial(wt)
    assert part[-8:] == (0).to_bytes(4, "little") + (1).to_bytes(4, "little")
    (a, b, c), _ = zkp_amd.proof_combine_raw(zk, [part], wt, r, s)
    assert {"A": a, "B": b, "C": c} == want
    assert p.prove_raw(wt, r, s)[0] == (a, b, c)


@pytest.mark.parametrize("name,nparts,balance", [("small", 2, False), ("small", 3, False), ("venmo_mini", 4, False),
                                                  ("venmo_mini", 5, True), ("small", 4, True)])
def test_split_distributed_quotient(name, nparts, balance, monkeypatch):
    # the distributed quotient on one GPU: part v % nparts extends vector v only
    # (zkp_quotient_part_staged), every part joins just its domain slice from the exchanged
    # slices (zkp_prove_partial_ext_staged); partials and proof stay bit-exact.  balance:
    # ZKP_SPLIT_BALANCE=1 weighted point slices (the quotient-vector owners take fewer points)
    import torch
    from zkp_amd.dist import split_range
    if balance:
        monkeypatch.setenv("ZKP_SPLIT_BALANCE", "1")
    zk, wt, r, s, want = _case(name)
    provers = [zkp_amd.Prover(zk, devices=[0], part=k, nparts=nparts) for k in range(nparts)]
    n = provers[0].domain_size
    full = [torch.empty(n * 32, dtype=torch.uint8, device="cuda") for _ in range(3)]
    for k, p in enumerate(provers):
        p.stage(wt, 0)
        mine = [v for v in range(3) if v % nparts == k]
        if mine:
            p.quotient_part_staged(0, sum(1 << v for v in mine),
                                   [full[v].data_ptr() if v in mine else None for v in range(3)])
    parts = []
    for k, p in enumerate(provers):
        lo, hi = split_range(n, k, nparts)
        sl = [full[v][lo * 32:hi * 32].clone() for v in range(3)]
        torch.cuda.synchronize()
        parts.append(p.prove_partial_ext_staged(0, [t.data_ptr() for t in sl]))
    for p in provers:
        p.close()
    assert parts == _oracle_partials(zk, wt, nparts, balance)
    (a, b, c), _ = zkp_amd.proof_combine_raw(zk, parts, wt, r, s)
    assert {"A": a, "B": b, "C": c} == want


@pytest.mark.parametrize("name", ["small", "venmo_mini", "synth_2^14"])
def test_batched_coset_extension_equals_per_vector(name):
    # zkp_quotient_part_staged extends the vectors of its mask in one launch per pass
    # (NttEngine::coset_extend_batch, workgroup w: tile w mod 2^lt of the w >> lt-th vector); every
    # mask must give the same bytes per vector as extending that vector alone
    import torch
    if name.startswith("synth"):  # full 1024-element tiles, 16 per vector
        from zkp_amd import synth
        circ = synth.Circuit(9000, (1 << 14) - 40, 5, 0x5A4B5032)
        zk, wt = circ.zkey(0x5A4B5033).bytes(), circ.witness(7)
    else:
        zk, wt, r, s, want = _case(name)
    p = zkp_amd.Prover(zk, devices=[0], part=0, nparts=1)
    try:
        n = p.domain_size
        p.stage(wt, 0)
        alone = []
        for v in range(3):
            t = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
            p.quotient_part_staged(0, 1 << v, [t.data_ptr() if u == v else None for u in range(3)])
            alone.append(t.cpu())
        for mask in (7, 5, 6, 3):
            out = [torch.full((n * 32,), 0xA5, dtype=torch.uint8, device="cuda") for _ in range(3)]
            p.quotient_part_staged(0, mask, [out[v].data_ptr() if mask >> v & 1 else None for v in range(3)])
            for v in range(3):
                if mask >> v & 1:
                    assert torch.equal(out[v].cpu(), alone[v]), (mask, v)
    finally:
        p.close()
