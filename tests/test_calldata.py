"""§8f row 3: calldata export + on-chain acceptance harness (no GPU).

zkp_proof_calldata (C ABI) and groth16.js exportSolidityCallData must both produce
snarkjs 0.4.22's `zkey export soliditycalldata` text (reference
circuit/scripts/generate_calldata.sh:3; format recalled from snarkjs: "0x" + 64 hex
digits, G2 pairs in EIP-197 [c1, c0] order -- pinned by Verifier.sol:184-188 and the
app's reformatProofForChain, SubmitOrderOnRampForm.tsx:36-46), and the restated
Verifier.sol must accept the golden proofs through that text."""
import json
import os
import shutil
import subprocess

import pytest

from oracle import binfile, groth16
import zkp_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
JS = os.path.join(ROOT, "zk-p2p-onramp_amd", "js")
NODE = shutil.which("node")
NAMES = ["tiny", "small", "venmo_mini"]


def _golden(name):
    proof = json.load(open(os.path.join(GOLD, "proof_%s.json" % name)))
    pub = json.load(open(os.path.join(GOLD, "public_%s.json" % name)))
    return proof, pub


def _expected(proof, pub):
    p = lambda n: '"0x%064x"' % int(n)
    a, b, c = proof["pi_a"], proof["pi_b"], proof["pi_c"]
    return ("[%s, %s]," % (p(a[0]), p(a[1])) +
            "[[%s, %s],[%s, %s]]," % (p(b[0][1]), p(b[0][0]), p(b[1][1]), p(b[1][0])) +
            "[%s, %s]," % (p(c[0]), p(c[1])) + "[%s]" % ",".join(p(x) for x in pub))


@pytest.mark.parametrize("name", NAMES)
def test_calldata_c_abi_and_acceptance(name):
    proof, pub = _golden(name)
    t = groth16.proof_from_json_obj(proof)
    cd = zkp_amd.solidity_calldata((t["A"], t["B"], t["C"]), [int(x) for x in pub])
    assert cd == _expected(proof, pub)
    z = binfile.read_zkey(open(os.path.join(GOLD, "circuit_%s.zkey" % name), "rb").read())
    assert groth16.verify_calldata(z, cd)
    if name == "tiny":  # a changed public input is rejected, an out-of-field one reverts
        bad = json.loads("[" + cd + "]")
        bad[3][0] = "0x%064x" % (int(bad[3][0], 16) + 1)
        assert not groth16.verify_calldata(z, json.dumps(bad)[1:-1])
        bad[3][0] = "0x%064x" % groth16.R
        assert not groth16.verify_calldata(z, json.dumps(bad)[1:-1])


@pytest.mark.skipif(NODE is None or not os.path.exists(os.path.join(JS, "build", "zkp_napi.node")),
                    reason="node or addon not available")
@pytest.mark.parametrize("name", ["small"])
def test_calldata_js_cli_and_onramp_args(name, tmp_path):
    proof, pub = _golden(name)
    pp = os.path.join(GOLD, "proof_%s.json" % name)
    pb = os.path.join(GOLD, "public_%s.json" % name)
    r = subprocess.run([NODE, os.path.join(JS, "cli.js"), "zkey", "export", "soliditycalldata", pb, pp],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == _expected(proof, pub)
    code = ("const z=require('./zk-p2p-onramp_amd/js/groth16.js');const fs=require('fs');"
            "const p=JSON.parse(fs.readFileSync(%r));const s=JSON.parse(fs.readFileSync(%r));"
            "console.log(JSON.stringify(z.onRampArgs(p,s)));" % (pp, pb))
    r = subprocess.run([NODE, "-e", code], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    a, b, c, sig = json.loads(r.stdout)
    assert a == proof["pi_a"][:2] and c == proof["pi_c"][:2] and sig == pub
    assert b == [proof["pi_b"][0][::-1], proof["pi_b"][1][::-1]]
