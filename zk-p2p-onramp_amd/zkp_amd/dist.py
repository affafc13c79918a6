"""Multi-GPU glue over torch.distributed (one process per GPU; backend "nccl" is RCCL
on ROCm, "gloo" for CPU tests).  Two scaling modes:

* replicas (batch of independent proofs): every rank owns a full resident zkey on its
  GPU and proves its own witnesses -- no collective on the data path
  (bench.py --gpus N, Prover.prove_batch inside one process).
* split (one large proof): rank k of G holds only point slice k of every section,
  computes its MSM partial sums (zkp_prove_partial, 392 bytes), and ONE all-gather of
  G x 392 bytes over xGMI brings every slice's partials to every rank, which sums them
  and assembles the proof on the host (zkp_proof_combine) -- bit-identical to the
  single-GPU proof.  The quotient H is computed in full by every rank.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import PARTIAL_BYTES, Prover, proof_combine_raw


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
        """Every rank returns the same proof tuple (as Prover.prove_raw).  r / s must be
        equal on all ranks (None draws them per rank: pass explicit values in production
        so that every rank assembles the same proof, or use rank 0's result)."""
        part = self.prover.prove_partial_staged(staged_slot) if staged_slot is not None else self.partial(wtns)
        parts = all_gather_partials(part, self.group)
        return proof_combine_raw(self.zkey, parts, wtns, r, s)
