"""GPU end-to-end parity: zkp_prove through the C ABI vs the oracle's golden
proofs at fixed r, s (bit-exact A, B, C), verification of random-r,s proofs,
batch mode, and snarkjs error behaviour."""
import json
import os
import struct

import pytest

from oracle import binfile, bn254, groth16
import zkp_amd

pytestmark = pytest.mark.gpu
NAMES = ["tiny", "small", "venmo_mini"]


def _files(golden_dir, name):
    zk = open(os.path.join(golden_dir, "circuit_%s.zkey" % name), "rb").read()
    wt = open(os.path.join(golden_dir, "circuit_%s.wtns" % name), "rb").read()
    return zk, wt


@pytest.mark.parametrize("name", NAMES)
def test_prove_bit_exact(golden_dir, name):
    zk, wt = _files(golden_dir, name)
    man = json.load(open(os.path.join(golden_dir, "manifest.json")))["circuits"][name]
    p = zkp_amd.Prover(zk)
    res = p.prove(wt, r=int(man["r"]), s=int(man["s"]))
    want_proof = open(os.path.join(golden_dir, "proof_%s.json" % name)).read()
    want_pub = open(os.path.join(golden_dir, "public_%s.json" % name)).read()
    assert groth16.js_stringify(res["proof"]) == want_proof
    assert groth16.js_stringify(res["publicSignals"]) == want_pub


# MSM tuning options (ZKP_MSM, read when the prover is built) and the serial profiling mode: other
# window bits and table depths (several bucket groups folded by Horner), task sizes, bucket-reduction
# segment sizes, every kernel alone on the device, the witness accumulations beside the G2 one from the
# start or only C after it (ZKP_G2FIRST) -- every variant must give the same golden proof
KNOBS = [{"ZKP_MSM": "seg=16"}, {"ZKP_MSM": "seg=2"}, {"ZKP_MSM": "task_w=24,task_h=48"},
         {"ZKP_MSM": "w=9,h=13"}, {"ZKP_MSM": "w=8,h=8,depth=3"}, {"ZKP_MSM": "w=20,h=20,depth=1"},
         {"ZKP_SERIAL": "1"}, {"ZKP_G2FIRST": "0"}, {"ZKP_G2FIRST": "3"}]


@pytest.mark.parametrize("knobs", KNOBS, ids=lambda k: ",".join("%s=%s" % kv for kv in k.items()))
@pytest.mark.parametrize("name", ["small", "venmo_mini"])
def test_prove_bit_exact_variants(golden_dir, name, knobs, monkeypatch):
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    zk, wt = _files(golden_dir, name)
    man = json.load(open(os.path.join(golden_dir, "manifest.json")))["circuits"][name]
    res = zkp_amd.Prover(zk).prove(wt, r=int(man["r"]), s=int(man["s"]))
    assert groth16.js_stringify(res["proof"]) == open(os.path.join(golden_dir, "proof_%s.json" % name)).read()


@pytest.mark.parametrize("name", NAMES)
def test_random_rs_verifies(golden_dir, name):
    zk, wt = _files(golden_dir, name)
    z = binfile.read_zkey(zk)
    (a, b, c), pub = zkp_amd.Prover(zk).prove_raw(wt)
    assert groth16.verify_with_zkey(z, pub, {"A": a, "B": b, "C": c})


def test_batch_matches_single(golden_dir):
    zk, wt = _files(golden_dir, "small")
    p = zkp_amd.Prover(zk)
    rs = [3, 5, 7]
    ss = [11, 13, 17]
    batch = p.prove_batch_raw([wt] * 3, rs, ss)
    for i in range(3):
        assert batch[i] == p.prove_raw(wt, rs[i], ss[i])


def test_groth16_module_api(golden_dir, tmp_path):
    zk, wt = _files(golden_dir, "tiny")
    zp = tmp_path / "c.zkey"
    wp = tmp_path / "w.wtns"
    zp.write_bytes(zk)
    wp.write_bytes(wt)
    man = json.load(open(os.path.join(golden_dir, "manifest.json")))["circuits"]["tiny"]
    out = zkp_amd.groth16.prove(str(zp), {"type": "mem", "data": wt}, r=int(man["r"]), s=int(man["s"]))
    assert groth16.js_stringify(out["proof"]) == open(os.path.join(golden_dir, "proof_tiny.json")).read()
    # CLI-equivalent file output
    p = zkp_amd.Prover(str(zp))
    p.prove_files(str(wp), str(tmp_path / "proof.json"), str(tmp_path / "public.json"))
    pj = json.load(open(tmp_path / "proof.json"))
    pub = [int(x) for x in json.load(open(tmp_path / "public.json"))]
    z = binfile.read_zkey(zk)
    assert groth16.verify_with_zkey(z, pub, groth16.proof_from_json_obj(pj))
    assert open(tmp_path / "public.json").read() == open(os.path.join(golden_dir, "public_tiny.json")).read()


@pytest.mark.parametrize("spec", ["w=7", "h=25", "depth=0", "seg=3", "nope=1", "w"])
def test_msm_options_rejected(golden_dir, monkeypatch, spec):
    """A malformed ZKP_MSM option fails the load with ZKP_ERR_INVALID_ARG instead of tuning nothing."""
    monkeypatch.setenv("ZKP_MSM", spec)
    zk, _ = _files(golden_dir, "tiny")
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.Prover(zk)
    assert e.value.status == 1 and ("ZKP_MSM" in e.value.message or "window bits" in e.value.message)


def test_errors(golden_dir):
    zk, wt = _files(golden_dir, "tiny")
    p = zkp_amd.Prover(zk)
    _, w = binfile.read_wtns(wt)
    with pytest.raises(zkp_amd.ZkpError) as e:
        p.prove(binfile.write_wtns(w + [5]))
    assert e.value.status == 6 and "Invalid witness length" in e.value.message
    bad = bytearray(wt)
    bad[0:4] = b"xxxx"
    with pytest.raises(zkp_amd.ZkpError) as e:
        p.prove(bytes(bad))
    assert e.value.status == 3
    # witness over a different prime -> curve mismatch
    sec1 = struct.pack("<I", 32) + bn254.int_to_le(bn254.P) + struct.pack("<I", len(w))
    sec2 = b"".join(bn254.int_to_le(x) for x in w)
    with pytest.raises(zkp_amd.ZkpError) as e:
        p.prove(binfile.write_binfile(b"wtns", 2, [(1, sec1), (2, sec2)]))
    assert e.value.status == 5


def test_gpu_proof_calldata_accepted(golden_dir):
    """GPU proof (random r, s) -> soliditycalldata -> restated Verifier.sol accepts it."""
    zk, wt = _files(golden_dir, "venmo_mini")
    z = binfile.read_zkey(zk)
    proof, pub = zkp_amd.Prover(zk).prove_raw(wt)
    assert groth16.verify_calldata(z, zkp_amd.solidity_calldata(proof, pub))


def test_prove_from_chunked_gz_zkey(golden_dir, tmp_path):
    """The app's circuit.zkey{b..k}.gz chunks load straight into the prover (§8f row 2)."""
    import gzip
    zk, wt = _files(golden_dir, "small")
    step = (len(zk) + 9) // 10
    for i, s in enumerate("bcdefghijk"):
        (tmp_path / ("circuit.zkey%s.gz" % s)).write_bytes(gzip.compress(zk[i * step:(i + 1) * step]))
    man = json.load(open(os.path.join(golden_dir, "manifest.json")))["circuits"]["small"]
    res = zkp_amd.Prover(str(tmp_path / "circuit.zkey")).prove(wt, r=int(man["r"]), s=int(man["s"]))
    assert groth16.js_stringify(res["proof"]) == open(os.path.join(golden_dir, "proof_small.json")).read()


def test_batch_per_proof_status(golden_dir):
    """zkp_prove_batch_status: a bad witness fails alone (its status), the rest prove."""
    zk, wt = _files(golden_dir, "small")
    _, bad = _files(golden_dir, "tiny")  # other circuit: wrong witness length
    p = zkp_amd.Prover(zk)
    res, st = p.prove_batch_status_raw([wt, bad, wt, b"garbage!" * 4], [3, 3, 5, 5], [7, 7, 9, 9])
    assert st == [0, 6, 0, 3]
    assert res[1] is None and res[3] is None
    assert res[0] == p.prove_raw(wt, 3, 7) and res[2] == p.prove_raw(wt, 5, 9)
    with pytest.raises(zkp_amd.ZkpError) as e:  # the all-or-error entry point reports the first failure
        p.prove_batch_raw([wt, bad], [3, 3], [7, 7])
    assert e.value.status == 6 and "proof 1" in e.value.message


def test_batch_requeues_on_device_failure(golden_dir, monkeypatch):
    """Two pipelines (both on device 0); the test hook makes pipeline 1 report a device failure
    on its second proof: its witness is re-queued to pipeline 0, every proof of the batch
    succeeds bit-exactly, and later single proofs skip the failed pipeline."""
    monkeypatch.setenv("ZKP_TEST_FAIL", "1:1")
    zk, wt = _files(golden_dir, "small")
    man = json.load(open(os.path.join(golden_dir, "manifest.json")))["circuits"]["small"]
    r, s = int(man["r"]), int(man["s"])
    p = zkp_amd.Prover(zk, devices=[0, 0])
    n = 12
    res, st = p.prove_batch_status_raw([wt] * n, [r] * n, [s] * n)
    assert st == [0] * n
    want = open(os.path.join(golden_dir, "proof_small.json")).read()
    for (a, b, c), _ in res:
        assert groth16.js_stringify(zkp_amd.proof_object(a, b, c)) == want
    for _ in range(3):  # round-robin now skips the failed pipeline
        assert groth16.js_stringify(p.prove(wt, r=r, s=s)["proof"]) == want


def test_concurrent_prove_on_one_handle(golden_dir):
    """Two host threads call zkp_prove on one handle at once (each takes an upload slot; the
    proofs run one at a time on the device): every result equals the sequential one."""
    import threading
    zk, wt = _files(golden_dir, "venmo_mini")
    p = zkp_amd.Prover(zk)
    want = {k: p.prove_raw(wt, 100 + k, 200 + k) for k in range(8)}
    got, errs = {}, []

    def run(ks):
        try:
            for k in ks:
                got[k] = p.prove_raw(wt, 100 + k, 200 + k)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)
    th = [threading.Thread(target=run, args=(range(i, 8, 2),)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs and got == want


def test_staged_concurrent_on_inflight_pipelines(golden_dir, monkeypatch):
    """ZKP_INFLIGHT=2: staged witnesses live in device 0's first pipeline; two host threads
    calling zkp_prove_staged at once take both pipelines (the second reads the witness in place).
    Every concurrent proof equals the golden proof."""
    import threading
    monkeypatch.setenv("ZKP_INFLIGHT", "2")
    zk, wt = _files(golden_dir, "venmo_mini")
    man = json.load(open(os.path.join(golden_dir, "manifest.json")))["circuits"]["venmo_mini"]
    r, s = int(man["r"]), int(man["s"])
    want = open(os.path.join(golden_dir, "proof_venmo_mini.json")).read()
    p = zkp_amd.Prover(zk)
    for slot in range(2):
        p.stage(wt, slot=slot)
    ref = p.prove_staged_raw(0, r, s)
    assert groth16.js_stringify(zkp_amd.proof_object(*ref[0])) == want
    out, errs = [], []

    def work(k):
        try:
            for i in range(6):
                out.append(p.prove_staged_raw((i + k) % 2, r, s))
        except BaseException as e:  # re-raised below
            errs.append(e)
    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    assert len(out) == 12 and all(o == ref for o in out)


@pytest.mark.parametrize("circuit", ["small", "venmo_mini"])
def test_batch_inflight_shared_tables(golden_dir, monkeypatch, circuit):
    """ZKP_INFLIGHT=3: three pipelines on device 0 share one copy of the base tables; a batch
    over them (several proofs in flight at once) and round-robin single proofs on each
    pipeline all reproduce the golden proof bit-exactly."""
    monkeypatch.setenv("ZKP_INFLIGHT", "3")
    zk, wt = _files(golden_dir, circuit)
    man = json.load(open(os.path.join(golden_dir, "manifest.json")))["circuits"][circuit]
    r, s = int(man["r"]), int(man["s"])
    p = zkp_amd.Prover(zk)
    want = open(os.path.join(golden_dir, "proof_%s.json" % circuit)).read()
    n = 9
    res, st = p.prove_batch_status_raw([wt] * n, [r] * n, [s] * n)
    assert st == [0] * n
    for (a, b, c), _ in res:
        assert groth16.js_stringify(zkp_amd.proof_object(a, b, c)) == want
    for _ in range(3):  # zkp_prove round-robins over the three pipelines
        assert groth16.js_stringify(p.prove(wt, r=r, s=s)["proof"]) == want
