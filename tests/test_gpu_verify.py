"""Verify-before-return on the GPU prover (SURVEY.md §5 failure detection; the reference runs
`snarkjs groth16 verify` right after every proof: dizkus-scripts/5_gen_proof.sh:14-21).

A silent device error is injected with the test hook ZKP_TEST_CORRUPT_H=1 (the H MSM result off
by one generator): with verification off the prover returns a proof that the restated
Verifier.sol rejects; with it on (zkp_prover_set_verify, or ZKP_VERIFY=1 at load) the proof is
never returned -- zkp_prove, zkp_prove_staged and every proof of a batch report ZKP_ERR_INTERNAL.
Healthy proofs pass the check unchanged (bit-exact golden proofs) and report its host cost.
The default (mode 2) checks every batch proof and no single proof: with ZKP_TEST_CORRUPT_H=2 (only
the odd-indexed proofs of a batch corrupted) the default batch refuses exactly those and proves
the rest."""
import json
import os

import pytest

from oracle import groth16
import zkp_amd

pytestmark = pytest.mark.gpu
ERR_INTERNAL = 9


def _case(golden_dir, name):
    zk = open(os.path.join(golden_dir, "circuit_%s.zkey" % name), "rb").read()
    wt = open(os.path.join(golden_dir, "circuit_%s.wtns" % name), "rb").read()
    man = json.load(open(os.path.join(golden_dir, "manifest.json")))["circuits"][name]
    want = open(os.path.join(golden_dir, "proof_%s.json" % name)).read()
    return zk, wt, int(man["r"]), int(man["s"]), want


@pytest.mark.parametrize("name", ["small", "venmo_mini"])
def test_verify_on_healthy_proofs_unchanged(golden_dir, name):
    zk, wt, r, s, want = _case(golden_dir, name)
    p = zkp_amd.Prover(zk)
    p.set_verify(True)
    res = p.prove(wt, r=r, s=s)
    assert groth16.js_stringify(res["proof"]) == want
    assert p.timings()["verify"] > 0
    batch = p.prove_batch_raw([wt] * 4, [r] * 4, [s] * 4)
    assert all(groth16.js_stringify(zkp_amd.proof_object(*x[0])) == want for x in batch)
    p.close()


def test_corrupt_device_result_is_caught(golden_dir, monkeypatch):
    monkeypatch.setenv("ZKP_TEST_CORRUPT_H", "1")
    zk, wt, r, s, want = _case(golden_dir, "venmo_mini")
    p = zkp_amd.Prover(zk)
    proof, pub = p.prove_raw(wt, r, s)  # verification off: the bad proof goes out ...
    assert not zkp_amd.proof_verify(zk, proof, pub)  # ... and the verifier rejects it
    p.set_verify(True)
    with pytest.raises(zkp_amd.ZkpError) as e:
        p.prove_raw(wt, r, s)
    assert e.value.status == ERR_INTERNAL and "verify-before-return" in e.value.message
    p.stage(wt, slot=0)
    with pytest.raises(zkp_amd.ZkpError) as e:
        p.prove_staged_raw(0, r, s)
    assert e.value.status == ERR_INTERNAL
    res, st = p.prove_batch_status_raw([wt] * 3, [r] * 3, [s] * 3)
    assert st == [ERR_INTERNAL] * 3 and res == [None] * 3
    p.close()


def test_verify_env_default(golden_dir, monkeypatch):
    monkeypatch.setenv("ZKP_VERIFY", "1")
    monkeypatch.setenv("ZKP_TEST_CORRUPT_H", "1")
    zk, wt, r, s, _ = _case(golden_dir, "small")
    p = zkp_amd.Prover(zk)
    with pytest.raises(zkp_amd.ZkpError) as e:
        p.prove_raw(wt, r, s)
    assert e.value.status == ERR_INTERNAL
    p.close()


def test_default_batch_refuses_corrupt_proves_rest(golden_dir, monkeypatch):
    monkeypatch.delenv("ZKP_VERIFY", raising=False)
    monkeypatch.setenv("ZKP_TEST_CORRUPT_H", "2")
    zk, wt, r, s, want = _case(golden_dir, "venmo_mini")
    p = zkp_amd.Prover(zk)
    assert p.verify_mode() == zkp_amd.Prover.VERIFY_BATCH
    res, st = p.prove_batch_status_raw([wt] * 6, [r] * 6, [s] * 6)
    assert st == [0, ERR_INTERNAL] * 3
    for i in (0, 2, 4):
        assert groth16.js_stringify(zkp_amd.proof_object(*res[i][0])) == want
    assert res[1] is None and res[3] is None and res[5] is None
    # single proofs are not checked by default (mode 2): a single proof is never corrupted by hook 2
    assert groth16.js_stringify(p.prove(wt, r=r, s=s)["proof"]) == want
    p.set_verify(False)
    res, st = p.prove_batch_status_raw([wt] * 2, [r] * 2, [s] * 2)
    assert st == [0, 0]  # verification off: the corrupted proof goes out unchecked ...
    assert not zkp_amd.proof_verify(zk, *res[1])  # ... and the verifier rejects it
    p.close()
