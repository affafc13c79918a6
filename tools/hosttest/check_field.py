#!/usr/bin/env python3
"""Drive tools/hosttest/field_host (device field/curve code compiled for the host)
with random inputs and compare against the Python oracle."""
import os, random, subprocess, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from oracle import bn254
P, R = bn254.P, bn254.R
RP = 1 << 261
BIN = os.environ.get("FIELD_HOST_BIN", os.path.join(os.path.dirname(__file__), "field_host"))

def w8(x): return " ".join("%x" % ((x >> (32 * i)) & 0xffffffff) for i in range(8))
def p8(s): return sum(int(t, 16) << (32 * i) for i, t in enumerate(s.split()[:8]))

def main(n=300):
    rnd = random.Random(1)
    lines, checks = [], []
    inv_rp_p = pow(RP, -1, P); inv_rp_r = pow(RP, -1, R)
    for _ in range(n):
        a, b = rnd.randrange(2 * P), rnd.randrange(2 * P)
        lines.append("mulq %s %s" % (w8(a), w8(b))); checks.append(("mulq", lambda v, a=a, b=b: v % P == a * b * inv_rp_p % P and v < 2 * P))
        lines.append("sqrq %s" % w8(a)); checks.append(("sqrq", lambda v, a=a: v % P == a * a * inv_rp_p % P and v < 2 * P))
        lines.append("addq %s %s" % (w8(a), w8(b))); checks.append(("addq", lambda v, a=a, b=b: v % P == (a + b) % P and v < 2 * P))
        lines.append("subq %s %s" % (w8(a), w8(b))); checks.append(("subq", lambda v, a=a, b=b: v % P == (a - b) % P and v < 2 * P))
        lines.append("canonq %s" % w8(a)); checks.append(("canonq", lambda v, a=a: v == a % P))
        x, y = rnd.randrange(2 * R), rnd.randrange(2 * R)
        lines.append("mulr %s %s" % (w8(x), w8(y))); checks.append(("mulr", lambda v, x=x, y=y: v % R == x * y * inv_rp_r % R and v < 2 * R))
    # lazy subtractions feeding multiplications (field.hpp lsub / rsub), incl. extremes
    edge = [0, 1, P - 1, P, P + 1, 2 * P - 1]
    # qreduce (add / sub / canon8 / canon4) at the extremes: a zero top limb against the largest
    # subtrahend (the wide-borrow top limb wraps), sums at 4m - 2, values just below multiples of m
    for a in edge + [(1 << 232) - 1, 1 << 232, 2 * P - (1 << 232)]:
        for b in edge + [(1 << 232) - 1]:
            lines.append("addq %s %s" % (w8(a), w8(b))); checks.append(("addq_edge", lambda v, a=a, b=b: v % P == (a + b) % P and v < 2 * P))
            lines.append("subq %s %s" % (w8(a), w8(b))); checks.append(("subq_edge", lambda v, a=a, b=b: v % P == (a - b) % P and v < 2 * P))
    # qreduce itself (Fr add / sub use it: FrCfg::QRED), incl. a zero top limb against the largest
    # subtrahend (the borrow form's top limb wraps) and values just below multiples of r
    edr = [0, 1, R - 1, R, R + 1, 2 * R - 1, (1 << 232) - 1, 1 << 232, 2 * R - (1 << 232)]
    for a in edr + [rnd.randrange(2 * R) for _ in range(n)]:
        for b in edr + [rnd.randrange(2 * R)]:
            lines.append("addr %s %s" % (w8(a), w8(b))); checks.append(("addr", lambda v, a=a, b=b: v % R == (a + b) % R and v < 2 * R))
            lines.append("subr %s %s" % (w8(a), w8(b))); checks.append(("subr", lambda v, a=a, b=b: v % R == (a - b) % R and v < 2 * R))
    for a in [0, 1, P, 2 * P - 1, 4 * P, 5 * P - 1, (1 << 256) - 1] + [rnd.randrange(1 << 256) for _ in range(n)]:
        lines.append("qredq %s" % w8(a)); checks.append(("qredq", lambda v, a=a: v % P == a % P and v < 6 * P // 5))
    pairs = [(rnd.randrange(2 * P), rnd.randrange(2 * P)) for _ in range(n)] + [(a, b) for a in edge for b in edge]
    for a, b in pairs:
        c = rnd.randrange(2 * P)
        lines.append("lsubmulq %s %s %s" % (w8(a), w8(b), w8(c)))
        checks.append(("lsubmulq", lambda v, a=a, b=b, c=c: v % P == (a - b) * c * inv_rp_p % P and v < 2 * P))
        lines.append("lsubsqrq %s %s" % (w8(a), w8(b)))
        checks.append(("lsubsqrq", lambda v, a=a, b=b: v % P == (a - b) * (a - b) * inv_rp_p % P and v < 2 * P))
        for cc in (c, 2 * P - 1):
            lines.append("rsubmulq %s %s %s" % (w8(a), w8(b), w8(cc)))
            checks.append(("rsubmulq", lambda v, a=a, b=b, c=cc: v % P == (a - b) * c * inv_rp_p % P and v < 2 * P))
        x, y, wv = a % (2 * R), b % (2 * R), rnd.randrange(2 * R)
        lines.append("rsubmulr %s %s %s" % (w8(x), w8(y), w8(wv)))
        checks.append(("rsubmulr", lambda v, x=x, y=y, w=wv: v % R == (x - y) * w * inv_rp_r % R and v < 2 * R))
    edge3 = [0, 1, P - 1, P, 2 * P - 1]
    triples = [(rnd.randrange(2 * P), rnd.randrange(2 * P), rnd.randrange(2 * P)) for _ in range(n)]
    triples += [(a, b, c) for a in edge3 for b in edge3 for c in edge3]
    for a, b, c in triples:
        lines.append("sub2xq %s %s %s" % (w8(a), w8(b), w8(c)))
        checks.append(("sub2xq", lambda v, a=a, b=b, c=c: v % P == (a - b - 2 * c) % P and v < 2 * P))
        x, y, z = a % (2 * R), b % (2 * R), c % (2 * R)
        lines.append("sub2xr %s %s %s" % (w8(x), w8(y), w8(z)))
        checks.append(("sub2xr", lambda v, x=x, y=y, z=z: v % R == (x - y - 2 * z) % R and v < 2 * R))
    # lazily reduced sums of products (field.hpp mul2): a, b < 4m; c, d <= 2m
    quads = [(rnd.randrange(4 * P), rnd.randrange(4 * P), rnd.randrange(2 * P + 1), rnd.randrange(2 * P + 1))
             for _ in range(n)]
    quads += [(4 * P - 1, 4 * P - 1, 2 * P, 2 * P), (0, 0, 0, 0), (4 * P - 1, 1, 2 * P, 2 * P - 1)]
    for a, b, c, d in quads:
        lines.append("mul2q %s %s %s %s" % (w8(a), w8(b), w8(c), w8(d)))
        checks.append(("mul2q", lambda v, a=a, b=b, c=c, d=d: v % P == (a * b + c * d) * inv_rp_p % P and v < 2 * P))
    # Fq2 products and sums of products (field.hpp Fq2 mul / mul2): components < 4m
    def f2(a0, a1, b0, b1):
        return (a0 * b0 - a1 * b1), (a0 * b1 + a1 * b0)
    f2cases = [[rnd.randrange(4 * P) for _ in range(8)] for _ in range(n)]
    f2cases += [[4 * P - 1] * 8, [0] * 8, [4 * P - 1, 0, 1, 4 * P - 1, 2 * P, 4 * P - 1, 4 * P - 1, 1]]
    for t in f2cases:
        lines.append("mulf2 %s" % " ".join(w8(x) for x in t[:4]))
        lines.append("mul2f2 %s" % " ".join(w8(x) for x in t))
        e = f2(*t[:4])
        g = f2(*t[4:])
        for k in range(2):
            checks.append(("mulf2", lambda v, x=e[k]: v % P == x * inv_rp_p % P and v < 2 * P))
        for k in range(2):
            checks.append(("mul2f2", lambda v, x=e[k] + g[k]: v % P == x * inv_rp_p % P and v < 2 * P))
    # NTT lazy radix-4 sums (field.hpp add_raw / add_raw_reduce / sub_raw6): inputs < 2m
    edge4 = [0, 1, R - 1, R, 2 * R - 1]
    r4 = [[rnd.randrange(2 * R) for _ in range(5)] for _ in range(n)]
    r4 += [[a, b, c, d, 2 * R - 1] for a in edge4 for b in edge4 for c in (0, 2 * R - 1) for d in (0, 2 * R - 1)]
    for x0, x1, x2, x3, wv in r4:
        lines.append("r4r %s" % " ".join(w8(x) for x in (x0, x1, x2, x3, wv)))
        s02, s13 = x0 + x2, x1 + x3
        checks.append(("r4r_sum", lambda v, t=s02 + s13: v % R == t % R and v < 2 * R))
        checks.append(("r4r_dif", lambda v, t=(s02 - s13) * wv: v % R == t * inv_rp_r % R and v < 2 * R))
    # Shoup product by a constant (field.hpp mul_shoup): a up to 2^261 with raw limbs < 2^31 (a borrow-
    # form difference), w < r plain, wq = floor(w 2^261 / r); result congruent and < 3r
    def l9(x, raw=False):
        if raw:  # limbs just below 2^31 where possible, same value: borrow 2^29 from each next limb
            limbs = [(x >> (29 * i)) & ((1 << 29) - 1) for i in range(9)]
            limbs[8] = x >> 232
            for i in range(8):
                if limbs[i + 1] >= 3:
                    limbs[i] += 3 << 29
                    limbs[i + 1] -= 3
            assert sum(v << (29 * i) for i, v in enumerate(limbs)) == x and max(limbs) < 1 << 31
        else:
            limbs = [(x >> (29 * i)) & ((1 << 29) - 1) for i in range(8)] + [x >> 232]
        return " ".join("%x" % v for v in limbs)
    sh = [(rnd.randrange(1 << 261), rnd.randrange(R)) for _ in range(n)]
    sh += [((1 << 261) - 1, R - 1), (0, R - 1), ((1 << 261) - 1, 1), (3 * R - 1, R - 1), (7 * R, R - 2), (1, 0)]
    for k, (a, wv) in enumerate(sh):
        wq = (wv << 261) // R
        lines.append("shoupr %s %s %s" % (l9(a, raw=k % 2 == 1), w8(wv), l9(wq)))
        checks.append(("shoupr", lambda z, a=a, wv=wv: z % R == a * wv % R and z < 3 * R))
    # round-5 NTT unit (ntt.hip r4_unit, field.hpp sub_raw6n): tile values < 3r normalised, at the value
    # extreme (3r - 1) and at the limb extreme (every low limb 2^29 - 1, top limb just below 3r's);
    # tw a table value < 2r (Montgomery), w a plain root < r with its Shoup quotient
    lowmax = (1 << 232) - 1
    x3e = [0, 1, 3 * R - 1, lowmax + ((((3 * R - 1) >> 232) - 1) << 232), lowmax, 2 * R - 1]
    twe = [2 * R - 1, lowmax + ((((2 * R - 1) >> 232) - 1) << 232), 1]
    quads4 = [[rnd.randrange(3 * R) for _ in range(4)] for _ in range(n)]
    quads4 += [[a, b, c, d] for a in x3e for b in x3e for c in x3e[2:4] for d in x3e[2:4]]
    quads4 += [[a, b, c, d] for a in x3e[2:4] for b in x3e[2:4] for c in x3e for d in x3e]
    # a small s02 against a maximal s13 (the top limb of s02 - s13 + 6m wrapped below zero)
    quads4 += [[a, b, c, d] for a in (0, 1) for c in (0, 1) for b in x3e[2:4] for d in x3e[2:4]]
    quads4 += [[b, a, d, c] for a in (0, 1) for c in (0, 1) for b in x3e[2:4] for d in x3e[2:4]]
    for k, (x0, x1, x2, x3) in enumerate(quads4):
        wv = R - 1 if k % 3 == 0 else rnd.randrange(R)
        tw = twe[k % 3] if k % 2 == 0 else rnd.randrange(2 * R)
        wq = (wv << 261) // R
        lines.append("r4lazy %s %s %s %s %s %s %s" % (w8(x0), w8(x1), w8(x2), w8(x3), w8(wv), l9(wq), w8(tw)))
        s02, s13 = x0 + x2, x1 + x3
        checks.append(("r4lazy_y1", lambda z, t=(s02 - s13) * wv: z % R == t % R and z < 3 * R))
        checks.append(("r4lazy_p1", lambda z, t=s02 - s13: z % R == t % R and z < 6 * R // 5))
        checks.append(("r4lazy_p0tw", lambda z, t=(s02 + s13) * tw: z % R == t * inv_rp_r % R and z < 2 * R))
        checks.append(("r4lazy_p1tw", lambda z, t=(s02 - s13) * tw: z % R == t * inv_rp_r % R and z < 2 * R))
        checks.append(("r4lazy_p2tw", lambda z, t=(x0 + x2) * tw: z % R == t * inv_rp_r % R and z < 2 * R))
        checks.append(("r4lazy_p3tw", lambda z, t=(x0 - x2) * tw: z % R == t * inv_rp_r % R and z < 2 * R))
        # the last pair's root w^0 (qreduce only) and the odd-b first radix-2 stage (ntt.hip, round 5)
        d02, d13 = x0 - x2, (x1 - x3) * wv
        checks.append(("r4last_d02", lambda z, t=d02: z % R == t % R and z < 6 * R // 5))
        checks.append(("r4last_p2", lambda z, t=d02 + d13: z % R == t % R and z < 6 * R // 5))
        checks.append(("r4last_p3", lambda z, t=d02 - d13: z % R == t % R and z < 6 * R // 5))
        checks.append(("r4last_p2tw", lambda z, t=(d02 + d13) * tw: z % R == t * inv_rp_r % R and z < 2 * R))
        checks.append(("r4last_p3tw", lambda z, t=(d02 - d13) * tw: z % R == t * inv_rp_r % R and z < 2 * R))
        checks.append(("r2first_sum", lambda z, t=x0 + x1: z % R == t % R and z < 6 * R // 5))
        checks.append(("r2first_dif", lambda z, t=(x0 - x1) * wv: z % R == t % R and z < 3 * R))
        checks.append(("shouptw_p0", lambda z, t=(s02 + s13) * wv: z % R == t % R and z < 3 * R))
        checks.append(("shouptw_p2", lambda z, t=(x0 + x2) * wv: z % R == t % R and z < 3 * R))
        checks.append(("shouptw_last_p2", lambda z, t=(d02 + d13) * wv: z % R == t % R and z < 3 * R))
        checks.append(("shouptw_last_p3", lambda z, t=(d02 - d13) * wv: z % R == t % R and z < 3 * R))
    # Shoup quotients of the NTT's stage roots (field.hpp shoup_quot) and sub4 against inputs < 4r
    RP_ = 1 << 261
    for wm in [0, 1, R - 1, R - 2] + [rnd.randrange(R) for _ in range(n)]:
        w = wm * pow(RP_, -1, R) % R
        lines.append("shoupq %s" % w8(wm))
        checks.append(("shoupq", lambda z, w=w: z == (w << 261) // R))
    for a in [0, 1, 3 * R - 1, 4 * R - 1, 2 * R] + [rnd.randrange(3 * R) for _ in range(n)]:
        for b in [0, 4 * R, 3 * R - 1, rnd.randrange(3 * R)]:
            lines.append("sub4r %s %s" % (w8(a), w8(b)))
            checks.append(("sub4r", lambda z, a=a, b=b: z % R == (a - b) % R and z < 2 * R))
    # lazily reduced G1 accumulator x (field.hpp sub_2x8 / lsub8 / canon8, curve.hpp acc_*): a, b, c
    # < 2m give x < 8m; consumers mul, sqr(lsub8), mul2 with an unnormalised rsub operand
    x8 = [[rnd.randrange(2 * P) for _ in range(4)] for _ in range(n)]
    x8 += [[a, b, c, d] for a in edge3 for b in edge3 for c in edge3 for d in (0, 2 * P - 1)]
    for a, b, c, d in x8:
        lines.append("x8q %s" % " ".join(w8(x) for x in (a, b, c, d)))
        x = a - b - 2 * c
        checks.append(("x8_canon", lambda v, x=x: v % P == x % P and v < 2 * P))
        checks.append(("x8_mul", lambda v, x=x, d=d: v % P == x * d * inv_rp_p % P and v < 2 * P))
        checks.append(("x8_lsub8_sqr", lambda v, x=x, d=d: v % P == (d - x) ** 2 * inv_rp_p % P and v < 2 * P))
        checks.append(("x8_mul2", lambda v, x=x, a=a, b=b, d=d: v % P == (d * (d - x) - a * b) * inv_rp_p % P
                       and v < 2 * P))
    # lazily reduced G2 accumulator forms (field.hpp sqr_lazy / sub_2x4, curve.hpp acc_y3):
    # inputs at the top of their bounds where 8 words can hold them (6m > 2^256: < 2^256 tested)
    TOP = (1 << 256) - 1
    def f2sq(a0, a1):
        return a0 * a0 - a1 * a1, 2 * a0 * a1
    sq = [[rnd.randrange(TOP), rnd.randrange(TOP)] for _ in range(n)] + [[TOP, TOP], [0, TOP], [TOP, 0], [0, 0]]
    for a0, a1 in sq:
        lines.append("sqrlazyf2 %s %s" % (w8(a0), w8(a1)))
        e = f2sq(a0, a1)
        for k in range(2):
            checks.append(("sqrlazyf2", lambda v, x=e[k]: v % P == x * inv_rp_p % P and v < 2 * P))
    for a, b, c in triples:
        t = [(a, b), (b, c), (c, a)]
        lines.append("sub2x4f2 %s" % " ".join(w8(x) for pr in t for x in pr))
        for k in range(2):
            x = t[0][k] - t[1][k] - 2 * t[2][k]
            checks.append(("sub2x4f2", lambda v, x=x: v % P == x % P and v < 4 * P))
    y3 = [[rnd.randrange(TOP), rnd.randrange(TOP), rnd.randrange(4 * P), rnd.randrange(4 * P),
           rnd.randrange(2 * P + 1), rnd.randrange(2 * P + 1), rnd.randrange(2 * P), rnd.randrange(2 * P)]
          for _ in range(n)]
    y3 += [[TOP, TOP, 4 * P - 1, 4 * P - 1, 2 * P, 2 * P, 2 * P - 1, 2 * P - 1], [0] * 8]
    for t0, t1, r0, r1, d0, d1, y0, y1 in y3:
        lines.append("y3f2 %s" % " ".join(w8(x) for x in (t0, t1, r0, r1, d0, d1, y0, y1)))
        c0 = t0 * r0 - t1 * r1 + d0 * y0 - d1 * y1
        c1 = t0 * r1 + t1 * r0 + d0 * y1 + d1 * y0
        for x in (c0, c1):
            checks.append(("y3f2", lambda v, x=x: v % P == x * inv_rp_p % P and v < 2 * P))
    for z in (0, P):
        lines.append("iszq %s" % w8(z)); checks.append(("iszq", lambda v: v == 1))
    out = subprocess.run([BIN], input="\n".join(lines) + "\n", capture_output=True, text=True).stdout.strip().split("\n")
    assert len(out) == len(checks), (len(out), len(checks))
    bad = {}
    for (name, fn), o in zip(checks, out):
        if name == "iszq":
            v = int(o)
        elif name == "shoupq":  # 9 limbs of 29 bits
            v = sum(int(t, 16) << (29 * i) for i, t in enumerate(o.split()[:9]))
        else:
            v = p8(o)
        if not fn(v):
            bad[name] = bad.get(name, 0) + 1
    print("checked", len(checks), "bad", bad)
    return not bad

if __name__ == "__main__":
    sys.exit(0 if main() else 1)

def curve_check(n=40):
    rnd = random.Random(2)
    inv_rp = pow(RP, -1, P)
    dev = lambda x: x * RP % P
    undev = lambda v: v * inv_rp % P
    lines, exp = [], []
    for i in range(n):
        p = bn254.g1_mul(bn254.G1_GEN, rnd.randrange(1, R))
        q = bn254.g1_mul(bn254.G1_GEN, rnd.randrange(1, R)) if i % 4 else p
        if i % 7 == 3:
            q = bn254.g1_neg(p)
        lines.append("g1add %s %s %s %s" % (w8(dev(p[0])), w8(dev(p[1])), w8(dev(q[0])), w8(dev(q[1]))))
        exp.append(("add", bn254.g1_add(p, q)))
        lines.append("g1addx %s %s %s %s" % (w8(dev(p[0])), w8(dev(p[1])), w8(dev(q[0])), w8(dev(q[1]))))
        exp.append(("addx", bn254.g1_add(p, bn254.g1_add(q, q))))
        z = rnd.randrange(P)
        lines.append("conv %s" % w8(z * (1 << 256) % P)); exp.append(("conv", z))
    out = subprocess.run([BIN], input="\n".join(lines) + "\n", capture_output=True, text=True).stdout.strip().split("\n")
    bad = 0
    for (kind, e), o in zip(exp, out):
        t = o.split()
        if kind == "conv":
            ok = undev(p8(" ".join(t[:8]))) == e
        else:
            X, Y, ZZ, ZZZ = [undev(p8(" ".join(t[8 * k:8 * k + 8]))) for k in range(4)]
            if ZZ == 0:
                got = None
            else:
                got = (X * pow(ZZ, -1, P) % P, Y * pow(ZZZ, -1, P) % P)
            ok = got == e
        if not ok:
            bad += 1
            print("BAD", kind)
    print("curve checked", len(exp), "bad", bad)
    return bad == 0

if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "curve":
    sys.exit(0 if curve_check() else 1)
