"""Multi-GPU glue over torch.distributed (one process per GPU; backend "nccl" is RCCL
on ROCm, "gloo" for CPU tests).  Two scaling modes:

* replicas (batch of independent proofs): every rank owns a full resident zkey on its
  GPU and proves its own witnesses -- no collective on the data path
  (bench.py --gpus N, Prover.prove_batch inside one process).
* split (one large proof): rank k of G holds only point slice k of every section,
  computes its MSM partial sums (zkp_prove_partial, 392 bytes), and ONE all-gather of
  G x 392 bytes over xGMI brings every slice's partials to every rank, which sums them
  and assembles the proof on the host (zkp_proof_combine) -- bit-identical to the
  single-GPU proof.  The quotient: either every rank computes it in full
  (SplitProver.prove_raw), or it is distributed (SplitProver.prove_raw_distq, SURVEY
  §8e E1(2)): rank v % G computes the coset extension of vector v in {A, B, C} and sends
  every rank the domain slice it needs (RCCL point-to-point over xGMI), so each rank only
  joins its own slice.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import PARTIAL_BYTES, Prover, proof_combine_raw


def split_range(n: int, part: int, nparts: int, balance=None):
    """[lo, hi) of slice `part` of n items cut into nparts contiguous ranges (as the C++
    split_range in prover.hip).  balance (default: ZKP_SPLIT_BALANCE=1 in the environment, which
    the C++ side reads too): for nparts > 3 the parts that extend a quotient vector (0..2) weigh
    max(1, 11 - nparts), the others 11."""
    if balance is None:
        balance = os.environ.get("ZKP_SPLIT_BALANCE") == "1"
    if not balance or nparts <= 3:
        return n * part // nparts, n * (part + 1) // nparts
    wq = max(1, 11 - nparts)  # see prover.hip split_range
    cum = lambda k: wq * min(k, 3) + 11 * max(k - 3, 0)  # noqa: E731
    return n * cum(part) // cum(nparts), n * cum(part + 1) // cum(nparts)


def exchange_quotient_slices(full, n: int, elem_bytes: int, group=None, device=None):
    """Redistribute the three quotient vectors A, B, C (n elements of elem_bytes each):
    rank v % G holds full[v] (a uint8 tensor of n * elem_bytes bytes; other entries are
    ignored); every rank receives its slice split_range(n, rank, G) of each vector.
    Owners send with batched point-to-point operations (no collective over the whole
    vector).  Returns [slice_A, slice_B, slice_C] as uint8 tensors on `device`."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    lo, hi = split_range(n, rank, world)
    out = [torch.empty((hi - lo) * elem_bytes, dtype=torch.uint8, device=device) for _ in range(3)]
    ops = []
    for v in range(3):
        owner = v % world
        if rank == owner:
            for k in range(world):
                klo, khi = split_range(n, k, world)
                sl = full[v][klo * elem_bytes:khi * elem_bytes]
                if k == rank:
                    out[v].copy_(sl)
                elif khi > klo:
                    ops.append(dist.P2POp(dist.isend, sl, dist.get_global_rank(group, k) if group else k, group))
        elif hi > lo:
            ops.append(dist.P2POp(dist.irecv, out[v], dist.get_global_rank(group, owner) if group else owner, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return out


def _gather_device(group):
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_gather_partials(part: bytes, group=None):
    """All-gather one zkp_partial per rank -> list of world_size partials (rank order).
    On "nccl" the exchange runs on the local GPU over RCCL (xGMI), on "gloo" on the CPU."""
    if len(part) != PARTIAL_BYTES:
        raise ValueError("a zkp_partial is %d bytes" % PARTIAL_BYTES)
    world = dist.get_world_size(group)
    dev = _gather_device(group)
    inp = torch.frombuffer(bytearray(part), dtype=torch.uint8).to(dev)
    out = torch.empty(world * PARTIAL_BYTES, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, inp, group=group)
    raw = out.cpu().numpy().tobytes()
    return [raw[i * PARTIAL_BYTES:(i + 1) * PARTIAL_BYTES] for i in range(world)]


def agree_blinding(r=None, s=None, group=None):
    """The blinding scalars every rank must use for one split proof: rank 0's r / s
    (drawn from the OS CSPRNG when None) broadcast to every rank, so all ranks assemble
    the SAME proof.  Explicit values are taken from rank 0 as well."""
    import secrets
    from . import R_MOD
    if dist.get_rank(group) == 0:
        vals = [int(r) % R_MOD if r is not None else secrets.randbelow(R_MOD),
                int(s) % R_MOD if s is not None else secrets.randbelow(R_MOD)]
    else:
        vals = [0, 0]
    src = dist.get_global_rank(group, 0) if group is not None else 0
    obj = [vals]
    dist.broadcast_object_list(obj, src=src, group=group)
    return obj[0][0], obj[0][1]


class SplitProver:
    """One proof split by point range over the ranks of `group` (one GPU per rank)."""

    def __init__(self, zkey, device: int, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.zkey = zkey
        self.prover = Prover(zkey, devices=[device], part=self.rank, nparts=self.world)

    def partial(self, wtns: bytes) -> bytes:
        return self.prover.prove_partial(wtns)

    def prove_raw(self, wtns: bytes, r=None, s=None, staged_slot=None):
        """Every rank returns the same proof tuple (as Prover.prove_raw): the blinding r / s
        is rank 0's (None = drawn once on rank 0 from the CSPRNG), broadcast to all ranks."""
        part = self.prover.prove_partial_staged(staged_slot) if staged_slot is not None else self.partial(wtns)
        parts = all_gather_partials(part, self.group)
        r, s = agree_blinding(r, s, self.group)
        return proof_combine_raw(self.zkey, parts, wtns, r, s)

    def prove_raw_distq(self, wtns: bytes, r=None, s=None, slot: int = 0, staged: bool = False):
        """As prove_raw, with the quotient distributed over the ranks (needs the "nccl"
        backend: the slices move between GPUs).  staged=True: the witness is already in
        `slot` (Prover.stage)."""
        if not staged:
            self.prover.stage(wtns, slot)
        n = self.prover.domain_size
        dev = torch.device("cuda", torch.cuda.current_device())
        mine = [v for v in range(3) if v % self.world == self.rank]
        full = [torch.empty(n * 32, dtype=torch.uint8, device=dev) if v in mine else None for v in range(3)]
        self.prover.quotient_part_staged(slot, sum(1 << v for v in mine),
                                         [t.data_ptr() if t is not None else None for t in full])
        sl = exchange_quotient_slices(full, n, 32, self.group, dev)
        torch.cuda.synchronize()
        part = self.prover.prove_partial_ext_staged(slot, [t.data_ptr() for t in sl])
        parts = all_gather_partials(part, self.group)
        r, s = agree_blinding(r, s, self.group)
        return proof_combine_raw(self.zkey, parts, wtns, r, s)
