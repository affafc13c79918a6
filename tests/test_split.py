"""Point-range split of ONE proof over several GPUs (SURVEY.md §8e E1(2), configs[4]):
host-side combine + the all-gather transport, without a GPU.

Partials here come from the oracle's restatement of the split (oracle.groth16.partial_sums);
zkp_proof_combine (host C code in libzkp_amd.so, no device) must turn any complete set
of them into the golden proof bit-exactly, and the gloo all-gather (world_size 2, the
same code path that runs over RCCL/xGMI with backend "nccl") must deliver them."""
import json
import os
import random
import socket

import pytest
import torch.multiprocessing as mp

from oracle import binfile, groth16
import zkp_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _case(name):
    zk = open(os.path.join(GOLD, "circuit_%s.zkey" % name), "rb").read()
    wt = open(os.path.join(GOLD, "circuit_%s.wtns" % name), "rb").read()
    man = json.load(open(os.path.join(GOLD, "manifest.json")))["circuits"][name]
    want = groth16.proof_from_json_obj(json.load(open(os.path.join(GOLD, "proof_%s.json" % name))))
    return zk, wt, int(man["r"]), int(man["s"]), want


def _oracle_partials(zk, wt, nparts, balance=False):
    z = binfile.read_zkey(zk)
    w = binfile.read_wtns(wt)[1]
    h = groth16.quotient_scalars(z, [x % groth16.R for x in w])
    out = []
    for k in range(nparts):
        p = groth16.partial_sums(z, w, k, nparts, h, balance)
        out.append(zkp_amd.partial_from_points(p["a"], p["b1"], p["c"], p["h"], p["b2"], k, nparts))
    return out


@pytest.mark.parametrize("name,nparts", [("tiny", 1), ("tiny", 3), ("small", 2), ("small", 7)])
def test_combine_oracle_partials_is_golden(name, nparts):
    zk, wt, r, s, want = _case(name)
    parts = _oracle_partials(zk, wt, nparts)
    random.Random(nparts).shuffle(parts)  # any order
    (a, b, c), pub = zkp_amd.proof_combine_raw(zk, parts, wt, r, s)
    assert {"A": a, "B": b, "C": c} == want
    assert pub == [x % groth16.R for x in binfile.read_wtns(wt)[1][1:len(pub) + 1]]


def test_combine_rejects_incomplete_or_duplicate_parts():
    zk, wt, r, s, _ = _case("tiny")
    parts = _oracle_partials(zk, wt, 3)
    for bad in (parts[:2], [parts[0], parts[0], parts[2]]):
        with pytest.raises(zkp_amd.ZkpError) as e:
            zkp_amd.proof_combine_raw(zk, bad, wt, r, s)
        assert e.value.status == 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, q):
    import torch.distributed as dist
    from zkp_amd.dist import all_gather_partials
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        zk, wt, r, s, _ = _case(name)
        mine = _oracle_partials(zk, wt, world)[rank]  # rank k computes slice k only
        parts = all_gather_partials(mine, None)
        (a, b, c), _ = zkp_amd.proof_combine_raw(zk, parts, wt, r, s)
        q.put((rank, [p[-8:] for p in parts], (a, b, c)))
    finally:
        dist.destroy_process_group()


def test_split_allgather_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(k, 2, port, "tiny", q)) for k in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    _, _, _, _, want = _case("tiny")
    for rank, tags, (a, b, c) in res:
        assert tags == [k.to_bytes(4, "little") + (2).to_bytes(4, "little") for k in range(2)]  # rank order
        assert {"A": a, "B": b, "C": c} == want


def _xchg_worker(rank, world, port, n, q, balance=False):
    import torch
    import torch.distributed as dist
    from zkp_amd.dist import exchange_quotient_slices, split_range
    if balance:
        os.environ["ZKP_SPLIT_BALANCE"] = "1"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def vec(v):  # deterministic stand-in for the coset evaluations of A, B, C
            g = torch.Generator().manual_seed(100 + v)
            return torch.randint(0, 256, (n * 32,), dtype=torch.uint8, generator=g)
        full = [vec(v) if v % world == rank else None for v in range(3)]
        got = exchange_quotient_slices(full, n, 32, None, torch.device("cpu"))
        lo, hi = split_range(n, rank, world)
        ok = all(torch.equal(got[v], vec(v)[lo * 32:hi * 32]) for v in range(3))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,balance", [(2, 64, False), (3, 50, False), (4, 37, False), (5, 101, True)])
def test_distributed_quotient_exchange_gloo(world, n, balance):
    # the slice exchange of the distributed quotient (zkp_amd.dist.exchange_quotient_slices,
    # RCCL point-to-point on GPUs): rank v % world owns vector v, every rank ends up with its
    # domain slice of all three, ragged slice sizes included
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xchg_worker, args=(k, world, port, n, q, balance)) for k in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res == {k: True for k in range(world)}


def _blind_worker(rank, world, port, q):
    import torch.distributed as dist
    from zkp_amd.dist import agree_blinding, all_gather_partials
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        zk, wt, _, _, _ = _case("tiny")
        parts = all_gather_partials(_oracle_partials(zk, wt, world)[rank], None)
        r, s = agree_blinding(None, None)  # production: no explicit r, s -> rank 0 draws them once
        (a, b, c), pub = zkp_amd.proof_combine_raw(zk, parts, wt, r, s)
        explicit = agree_blinding(7 + rank, 11 + rank)  # explicit values: rank 0's win
        q.put((rank, (r, s), (a, b, c), pub, explicit))
    finally:
        dist.destroy_process_group()


def test_split_blinding_agreed_gloo_world2():
    """SplitProver with r = s = None: every rank assembles the SAME (verifying) proof,
    because the blinding is drawn on rank 0 and broadcast (zkp_amd.dist.agree_blinding)."""
    from oracle import binfile, groth16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_blind_worker, args=(k, 2, port, q)) for k in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, rs0, pr0, pub0, ex0), (_, rs1, pr1, pub1, ex1) = res
    assert rs0 == rs1 and pr0 == pr1 and ex0 == ex1 == (7, 11)
    zk, _, _, _, _ = _case("tiny")
    a, b, c = pr0
    assert groth16.verify_with_zkey(binfile.read_zkey(zk), pub0, {"A": a, "B": b, "C": c})


@pytest.mark.parametrize("balance", [False, True])
def test_split_ranges_agree(balance):
    # zkp_amd.dist.split_range (the exchange, the emulation) and the oracle's (partial sums) give
    # the same contiguous tiling of [0, n) -- the C++ split_range is checked against them through
    # the GPU split tests; balanced: parts 0..2 weigh max(1, 11 - G), the others 11 (nparts > 3)
    from zkp_amd.dist import split_range
    for n in (1, 7, 100, 1 << 21, 6_400_562):
        for nparts in range(1, 10):
            rs = [split_range(n, k, nparts, balance) for k in range(nparts)]
            assert rs == [groth16.split_range(n, k, nparts, balance) for k in range(nparts)]
            assert rs[0][0] == 0 and rs[-1][1] == n and all(rs[k][1] == rs[k + 1][0] for k in range(nparts - 1))
            if balance and nparts > 3 and n >= 1 << 21:  # weights max(1, 11 - G) : 11
                wq = max(1, 11 - nparts)
                assert abs((rs[0][1] - rs[0][0]) * 11 - (rs[3][1] - rs[3][0]) * wq) <= 11 * 11
