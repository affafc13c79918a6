#!/usr/bin/env python3
"""Extract the DATA the reference holds for this path into tests/golden/reference_fixtures.json
(run once in the build container, where /root/reference exists; tests read only the JSON):

* app/src/helpers/vkey.ts:1-219      — the snarkjs verification key object (nPublic 26,
                                        alpha/beta/gamma/delta, vk_alphabeta_12, 27 IC points)
* contracts/Verifier.sol:33-36,52     — G2 generator (Solidity [c1,c0] order), base field p
* contracts/Verifier.sol:178-338      — Solidity verifying key (alfa1, beta2, gamma2, delta2, IC[27])
* contracts/Verifier.sol:341          — scalar field r
* test/ramp.test.js:193-196           — the hard-coded proof (a, b, c) and 26 public signals
* circuit/input.json                  — modulus / order_id / claim_id (public-signal layout)
"""
import json
import os
import re

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_fixtures.json")


def read(p):
    with open(os.path.join(REF, p)) as f:
        return f.read()


def vkey_ts():
    s = read("app/src/helpers/vkey.ts")
    body = s[s.index("{"):s.rindex("}") + 1]
    return json.loads(body)


def verifier_sol():
    s = read("contracts/Verifier.sol")
    nums = lambda t: [int(x) for x in re.findall(r"\d{5,}", t)]
    out = {}
    p2 = s[s.index("function P2()"):s.index("/*", s.index("function P2()"))]
    out["g2_generator_sol_order"] = nums(p2)  # [x.c1, x.c0, y.c1, y.c0]
    out["q"] = int(re.search(r"uint q = (\d+);", s).group(1))
    out["snark_scalar_field"] = int(re.search(r"uint256 snark_scalar_field = (\d+);", s).group(1))
    vk = s[s.index("function verifyingKey()"):s.index("function verify(")]
    out["alfa1"] = nums(vk[vk.index("vk.alfa1"):vk.index("vk.beta2")])
    out["beta2_sol_order"] = nums(vk[vk.index("vk.beta2"):vk.index("vk.gamma2")])
    out["gamma2_sol_order"] = nums(vk[vk.index("vk.gamma2"):vk.index("vk.delta2")])
    out["delta2_sol_order"] = nums(vk[vk.index("vk.delta2"):vk.index("vk.IC = ")])
    ic = []
    for m in re.finditer(r"vk\.IC\[(\d+)\] = Pairing\.G1Point\(\s*(\d+),\s*(\d+)\s*\);", vk):
        ic.append([int(m.group(2)), int(m.group(3))])
    out["IC"] = ic
    return out


def ramp_test():
    s = read("test/ramp.test.js")
    grab = lambda name: json.loads(re.search(r"let %s = (\[.*?\]);" % name, s).group(1).replace("'", '"'))
    return {"a": grab("a"), "b": grab("b"), "c": grab("c"), "signals": grab("signals")}


def main():
    inp = json.loads(read("circuit/input.json"))
    data = {
        "_source": "extracted by tests/golden/extract_reference_fixtures.py from the reference snapshot",
        "vkey_ts": vkey_ts(),
        "verifier_sol": {k: (str(v) if isinstance(v, int) else v) for k, v in verifier_sol().items()},
        "ramp_test_proof": ramp_test(),
        "input_json": {"modulus": inp["modulus"], "order_id": inp["order_id"], "claim_id": inp["claim_id"]},
    }
    # ints inside lists -> decimal strings for JSON portability
    def fix(o):
        if isinstance(o, list):
            return [fix(x) for x in o]
        if isinstance(o, dict):
            return {k: fix(v) for k, v in o.items()}
        if isinstance(o, int) and not isinstance(o, bool) and o > 2 ** 53:
            return str(o)
        return o
    with open(OUT, "w") as f:
        json.dump(fix(data), f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
