"""The C++ CPU restatement (oracle/cpu, used as checker + cpu_baseline) agrees
with the Python oracle on every golden vector."""
import json
import os
import subprocess

import pytest

from oracle import bn254, groth16

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def co():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from oracle import cpu_oracle
    return cpu_oracle


@pytest.mark.parametrize("name", ["tiny", "small", "venmo_mini"])
def test_cpu_port_proofs(co, name):
    man = json.load(open(os.path.join(GOLD, "manifest.json")))["circuits"][name]
    zk = open(os.path.join(GOLD, "circuit_%s.zkey" % name), "rb").read()
    wt = open(os.path.join(GOLD, "circuit_%s.wtns" % name), "rb").read()
    (a, b, c), _ = co.prove(zk, wt, int(man["r"]), int(man["s"]), threads=4)
    want = groth16.proof_from_json_obj(json.load(open(os.path.join(GOLD, "proof_%s.json" % name))))
    assert (a, b, c) == (want["A"], want["B"], want["C"])


@pytest.mark.parametrize("n", [64, 1024])
def test_cpu_port_msm_g1(co, n):
    blob = open(os.path.join(GOLD, "msm_g1_%d.bin" % n), "rb").read()
    e = blob[n * 96:]
    assert co.msm_g1(blob[:n * 64], blob[n * 64:n * 96], threads=4) == (bn254.le_to_int(e[:32]), bn254.le_to_int(e[32:]))


def test_cpu_port_msm_g2(co):
    n = 64
    blob = open(os.path.join(GOLD, "msm_g2_%d.bin" % n), "rb").read()
    e = blob[n * 160:]
    v = [bn254.le_to_int(e[32 * i:32 * i + 32]) for i in range(4)]
    assert co.msm_g2(blob[:n * 128], blob[n * 128:n * 160], threads=4) == ((v[0], v[1]), (v[2], v[3]))


@pytest.mark.parametrize("k", [1, 4, 10, 12])
def test_cpu_port_ntt_golden(co, k):
    """The standalone NTT export (g16cpu_ntt, the checker of the 2^20 / 2^23 GPU NTT tests) against the
    golden vectors: forward, inverse and coset extension."""
    d = json.load(open(os.path.join(GOLD, "ntt_%d.json" % k)))
    raw = b"".join(int(x).to_bytes(32, "little") for x in d["input"])

    def dec(b):
        return [bn254.le_to_int(b[32 * i:32 * i + 32]) for i in range(len(b) // 32)]
    for mode, key in ((0, "forward"), (1, "inverse"), (2, "coset")):
        assert dec(co.ntt(raw, mode, threads=4)) == [int(x) for x in d[key]], key


def test_cpu_port_ntt_rejects_bad_sizes(co):
    with pytest.raises(ValueError):
        co.ntt(b"\0" * 96, 0)
    with pytest.raises(ValueError):
        co.ntt(b"\0" * 64, 3)
