"""Compare tools/hosttest/msm_emu (the MSM kernels replayed on the host) with the oracle."""
import os, sys, subprocess, random
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."); os.chdir(ROOT); sys.path.insert(0, ROOT)
from oracle import bn254, groth16, circuit
R = bn254.R
rng = circuit.SplitMix64(7, 0)
g = bn254.FixedBase(bn254.G1_GEN)
def run(pts, sc, c=0, d=0, tag="", bal=0):
    blob = b"".join(bn254.g1_to_lem(p) for p in pts) + b"".join(bn254.int_to_le(x) for x in sc)
    open("/tmp/emu.bin", "wb").write(blob)
    out = subprocess.run(["tools/hosttest/msm_emu", "g1", "/tmp/emu.bin", str(len(pts)), str(c), str(d), str(bal)], capture_output=True, text=True).stdout.strip()
    want = groth16.msm_g1(pts, [x % R for x in sc])
    got = None if out == "inf" else tuple(int(v) for v in out.split())
    print(tag, c, d, bal, "OK" if got == want else "BAD", flush=True)
pts = [g.mul(rng.fr() or 1) for _ in range(200)]
sc = [rng.fr() for _ in range(200)]
for c, d in [(0, 0), (0, 1), (5, 0), (5, 3), (8, 7), (13, 0), (2, 0)]:
    run(pts, sc, c, d, "uniform")
for c in (0, 6, 8, 13):  # balanced window widths (c and c-1 bits; the H plan's option)
    run(pts, sc, c, 0, "balanced", 1)
run(pts, [R - 1 - i for i in range(200)], 13, 0, "balanced_top", 1)
run(pts, [1] * 200, 0, 0, "ones")
run(pts, [sum(1 << (8 * w) for w in range(31))] * 200, 8, 0, "alldigit1")
run(pts[:8], [R + 5, 2 * R + 1, (1 << 256) - 1, R, R - 1, 1, 2, 3], 0, 0, "above_r")
run([pts[0]] * 100, list(range(1, 101)), 0, 0, "same_point")
pts2 = pts[:50] + [None] * 3
# G2

def run2(pts, sc, c=0, d=0, tag="", bal=0):
    blob = b"".join(bn254.g2_to_lem(p) for p in pts) + b"".join(bn254.int_to_le(x) for x in sc)
    open("/tmp/emu2.bin", "wb").write(blob)
    out = subprocess.run(["tools/hosttest/msm_emu", "g2", "/tmp/emu2.bin", str(len(pts)), str(c), str(d), str(bal)], capture_output=True, text=True).stdout.strip()
    want = groth16.msm_g2(pts, [x % R for x in sc])
    v = None if out == "inf" else [int(t) for t in out.split()]
    got = None if v is None else ((v[0], v[1]), (v[2], v[3]))
    print("g2", tag, c, d, bal, "OK" if got == want else "BAD", flush=True)
p2 = [bn254.g2_mul(bn254.G2_GEN, rng.fr() or 1) for _ in range(24)]
run2(p2, [rng.fr() for _ in range(24)], 6, 0, "uniform")
run2(p2, [rng.fr() for _ in range(24)], 5, 3, "groups")
run2(p2, [rng.fr() for _ in range(24)], 6, 0, "balanced", 1)
run2([p2[0]] * 10, list(range(1, 11)), 4, 0, "same_point")
