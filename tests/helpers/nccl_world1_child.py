"""Child process of tests/test_gpu_nccl.py: initialise torch.distributed with backend "nccl" (RCCL) at
world size 1 on cuda:0 BEFORE any other GPU work in this process, then run zkp_amd.dist.SplitProver's
prove_raw (RCCL all-gather of the 392-byte partials + broadcast of the blinding) and prove_raw_distq
(RCCL slice exchange of the distributed quotient) on the golden circuits.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "zk-p2p-onramp_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    port = int(sys.argv[1])
    names = sys.argv[2:]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    out = {"backend": dist.get_backend(), "world": dist.get_world_size(), "cases": {}}
    try:
        from test_split import _case
        from zkp_amd.dist import SplitProver, all_gather_partials
        for name in names:
            zk, wt, r, s, want = _case(name)
            sp = SplitProver(zk, 0)
            (a, b, c), _ = sp.prove_raw(wt, r, s)
            ok_full = {"A": a, "B": b, "C": c} == want
            (a2, b2, c2), _ = sp.prove_raw_distq(wt, r, s, slot=0)
            ok_distq = {"A": a2, "B": b2, "C": c2} == want
            part = sp.partial(wt)
            ok_gather = all_gather_partials(part) == [part]
            sp.prover.close()
            out["cases"][name] = {"prove_raw": ok_full, "prove_raw_distq": ok_distq, "all_gather": ok_gather}
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
