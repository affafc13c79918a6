"""The RCCL code path of the split proof (zkp_amd.dist) on the one GPU available:
torch.distributed with backend "nccl" at world size 1, initialised in a fresh child process before any
other GPU work there (tests/helpers/nccl_world1_child.py).  SplitProver.prove_raw (all-gather of the
partials, blinding broadcast) and prove_raw_distq (distributed quotient, slice exchange) must give the
golden proofs.  Multi-rank RCCL stays unmeasured: no multi-GPU node."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_split_prover_over_rccl_world1():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(HERE, "helpers", "nccl_world1_child.py"), str(_free_port()),
                        "small", "venmo_mini"], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.returncode, p.stderr[-3000:])
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["cases"] == {name: {"prove_raw": True, "prove_raw_distq": True, "all_gather": True}
                            for name in ("small", "venmo_mini")}
