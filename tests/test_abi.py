"""C-ABI checks that need no GPU: the library loads, exports every symbol that
include/*.h declares, validates inputs before touching a device, and formats
snarkjs JSON byte-identically."""
import ctypes
import json
import os
import re
import struct

import pytest

import zkp_amd
from zkp_amd import synth
from oracle import binfile, bn254, circuit, groth16

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zkp_[a-z0-9_]+)\s*\(", src)))


@pytest.mark.parametrize("header,lib", [("zkp_amd.h", zkp_amd.LIB_PATH), ("zkp_synth.h", synth.LIB_PATH)])
def test_exports_every_declared_symbol(header, lib):
    names = _declared(header)
    assert len(names) > 5
    L = ctypes.CDLL(lib)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_version_and_error_before_device():
    assert "gfx950" in zkp_amd.version()
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.Prover(b"xxxx" + bytes(100))
    assert e.value.status == 3 and "Invalid File format" in e.value.message
    zk = bytearray(open(os.path.join(GOLD, "circuit_tiny.zkey"), "rb").read())
    # section 1 payload (protocol) lives right after the first section header (file header 12 + 12)
    proto = bytearray(zk)
    proto[24:28] = struct.pack("<I", 2)
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.Prover(bytes(proto))
    assert e.value.status == 4 and "not groth16" in e.value.message
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.Prover(bytes(zk[:len(zk) - 100]))
    assert e.value.status == 3
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.ntt_fr([1, 2, 3], 0)
    assert e.value.status == 1
    for count in (0, 4):  # the batched coset extension takes 1..3 vectors
        with pytest.raises(zkp_amd.ZkpError) as e:
            zkp_amd.bench_ntt(10, count=count)
        assert e.value.status == 1


def test_proof_json_formatting_matches_snarkjs():
    lib = zkp_amd.load_library()
    proof = groth16.proof_from_json_obj(json.load(open(os.path.join(GOLD, "proof_small.json"))))
    pub = [int(x) for x in json.load(open(os.path.join(GOLD, "public_small.json")))]
    pr = zkp_amd._Proof()
    le = lambda x: (ctypes.c_uint8 * 32)(*x.to_bytes(32, "little"))
    pr.pi_a[0], pr.pi_a[1] = le(proof["A"][0]), le(proof["A"][1])
    pr.pi_b[0][0], pr.pi_b[0][1] = le(proof["B"][0][0]), le(proof["B"][0][1])
    pr.pi_b[1][0], pr.pi_b[1][1] = le(proof["B"][1][0]), le(proof["B"][1][1])
    pr.pi_c[0], pr.pi_c[1] = le(proof["C"][0]), le(proof["C"][1])
    buf = (ctypes.c_uint8 * (32 * len(pub)))(*b"".join(x.to_bytes(32, "little") for x in pub))
    pr.n_public = pr.public_capacity = len(pub)
    pr.public_signals = ctypes.cast(buf, ctypes.POINTER(ctypes.c_uint8))
    out = ctypes.create_string_buffer(8192)
    need = ctypes.c_size_t()
    assert lib.zkp_proof_json(ctypes.byref(pr), out, 8192, ctypes.byref(need)) == 0
    assert out.value.decode() == open(os.path.join(GOLD, "proof_small.json")).read()
    assert lib.zkp_public_json(ctypes.byref(pr), out, 8192, ctypes.byref(need)) == 0
    assert out.value.decode() == open(os.path.join(GOLD, "public_small.json")).read()


def test_synth_witness_matches_oracle():
    c = synth.Circuit(300, 320, 26, 77)
    r1cs, w = circuit.gen_circuit(300, 320, 26, 77, wseed=5)
    assert c.witness(5) == binfile.write_wtns(w)
    assert circuit.check_witness(r1cs, w)


@pytest.mark.parametrize("bool_pct", [0, 30, 100])
def test_synth_witness_mix_matches_oracle(bool_pct):
    """The witness-mix knob (share of bit-valued AND/XOR steps) of the C++ generator is
    the oracle's, and the witness still satisfies the circuit."""
    c = synth.Circuit(300, 320, 26, 78, bool_pct=bool_pct)
    r1cs, w = circuit.gen_circuit(300, 320, 26, 78, wseed=6, bool_pct=bool_pct)
    assert c.witness(6) == binfile.write_wtns(w)
    assert circuit.check_witness(r1cs, w)
    if bool_pct == 0:  # only the free inputs (5 %), w0 and the public values are small
        assert sum(1 for x in w if x > 1) > 0.85 * len(w)
