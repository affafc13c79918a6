"""Seeded synthetic satisfiable R1CS ("Venmo-shaped") — TEST INFRASTRUCTURE ONLY.

The real Venmo circuit artefacts (.r1cs/.zkey/.wtns, circuit.wasm) are absent
(reference ``.gitignore:2-3,7,12,30``, ``.MISSING_LARGE_BLOBS:1``), so parity and
benchmarks run on synthetic circuits with the Venmo circuit's *shape*
(SURVEY.md §8d D2): nVars, nConstraints, nPublic, ~3 A+B coefficients per
constraint, and a witness that is mostly bits like a SHA/regex circuit
(``circuit/circuit.circom:62-134``).  The witness distribution is an ASSUMPTION.

Construction (mirrored bit-for-bit by the C++ generator
``zk-p2p-onramp_amd/csrc/synth/synth.hip`` — tests compare the two): the circuit
STRUCTURE comes from stream 3 of ``seed``; the witness's free inputs from stream 4
of ``wseed``, so many distinct witnesses share one circuit (batch benchmarks).

* w0 = 1; public w1..w_nPublic = random u64 values (packed-limb-like).
* the first ``n_in`` private signals are free input bits.
* every later private signal v is defined by ONE constraint, chosen by
  ``x = next() % 100``:
    x < 35  AND : (w_a)(w_b) = w_v                       a, b random bits
    x < 70  XOR : (2 w_a)(w_b) = w_a + w_b - w_v          a, b random bits
    else    MUL : (c1 w_a + c2 w_b)(c3 w_c + c4 w_0) = w_v  a, b, c < v, c_i random Fr
* remaining constraints are booleanity checks (w_b)(w_b - w_0) = 0, first
  over the input bits, then over random bits.
"""
from __future__ import annotations

from dataclasses import dataclass

from .bn254 import R

MASK64 = (1 << 64) - 1


class SplitMix64:
    """SplitMix64; stream s of seed k starts at state k + s * 0x632BE59BD9B4E019."""

    def __init__(self, seed: int, stream: int = 0):
        self.state = (seed + stream * 0x632BE59BD9B4E019) & MASK64

    def next(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def fr(self) -> int:
        """Uniform in [0, r): four LE u64 limbs, top limb masked to 62 bits, rejection-sampled."""
        while True:
            v = 0
            for i in range(4):
                v |= self.next() << (64 * i)
            v &= (1 << 254) - 1
            if v < R:
                return v

    def below(self, k: int) -> int:
        return self.next() % k


@dataclass
class R1CS:
    n_vars: int
    n_public: int
    n_constraints: int
    # each constraint: (A, B, C) with each a list of (signal, coef) sorted by signal
    constraints: list

    def coef_count_ab(self) -> int:
        return sum(len(a) + len(b) for a, b, _ in self.constraints)


def _lc(pairs):
    d = {}
    for s, c in pairs:
        d[s] = (d.get(s, 0) + c) % R
    return sorted((s, c) for s, c in d.items() if c != 0)


def gen_program(n_vars: int, n_constraints: int, n_public: int, seed: int, in_permille: int = 50,
                bool_pct: int = 70):
    """Circuit STRUCTURE from stream 3 of ``seed``: (R1CS, program).  program is the
    list of defining steps used by ``gen_witness``; nothing here depends on values.
    ``bool_pct``: share (percent) of AND/XOR (bit-valued) steps, the witness-mix knob;
    70 is the default assumption, 0 makes every defined signal a uniform MUL value."""
    rng = SplitMix64(seed, 3)
    n_priv = n_vars - 1 - n_public
    n_in = max(2, n_priv * in_permille // 1000)
    if n_priv < n_in:
        raise ValueError("too few private signals")
    bits = [1 + n_public + k for k in range(n_in)]
    cons = []
    prog = []
    for v in range(1 + n_public + n_in, n_vars):
        x = rng.below(100)
        if x < bool_pct:
            a = bits[rng.below(len(bits))]
            b = bits[rng.below(len(bits))]
            if x < bool_pct // 2:
                prog.append((0, a, b))
                cons.append((_lc([(a, 1)]), _lc([(b, 1)]), _lc([(v, 1)])))
            else:
                prog.append((1, a, b))
                cons.append((_lc([(a, 2)]), _lc([(b, 1)]), _lc([(a, 1), (b, 1), (v, R - 1)])))
            bits.append(v)
        else:
            a = rng.below(v)
            b = rng.below(v)
            c = rng.below(v)
            c1, c2, c3, c4 = rng.fr(), rng.fr(), rng.fr(), rng.fr()
            prog.append((2, a, b, c, c1, c2, c3, c4))
            cons.append((_lc([(a, c1), (b, c2)]), _lc([(c, c3), (0, c4)]), _lc([(v, 1)])))
    if len(cons) > n_constraints:
        raise ValueError("n_constraints too small for n_vars")
    i = 0
    while len(cons) < n_constraints:
        b = bits[i] if i < n_in else bits[rng.below(len(bits))]
        i += 1
        cons.append((_lc([(b, 1)]), _lc([(b, 1), (0, R - 1)]), []))
    meta = {"n_public": n_public, "n_in": n_in}
    return R1CS(n_vars, n_public, n_constraints, cons), (meta, prog)


def gen_witness(program, wseed: int):
    """Witness from stream 4 of ``wseed``: public values (u64) and input bits are
    free; every other signal is computed by its defining constraint."""
    meta, prog = program
    rng = SplitMix64(wseed, 4)
    w = [1]
    for _ in range(meta["n_public"]):
        w.append(rng.next())
    for _ in range(meta["n_in"]):
        w.append(rng.next() & 1)
    for step in prog:
        if step[0] == 0:
            w.append(w[step[1]] * w[step[2]])
        elif step[0] == 1:
            a, b = w[step[1]], w[step[2]]
            w.append((a + b - 2 * a * b) % R)
        else:
            _, a, b, c, c1, c2, c3, c4 = step
            w.append((c1 * w[a] + c2 * w[b]) * (c3 * w[c] + c4) % R)
    return w


def gen_circuit(n_vars: int, n_constraints: int, n_public: int, seed: int, in_permille: int = 50, wseed=None,
                bool_pct: int = 70):
    """Returns (R1CS, witness); the witness uses ``wseed`` (default: ``seed``)."""
    r1cs, prog = gen_program(n_vars, n_constraints, n_public, seed, in_permille, bool_pct)
    return r1cs, gen_witness(prog, seed if wseed is None else wseed)


def check_witness(r1cs: R1CS, w) -> bool:
    def ev(lc):
        return sum(c * w[s] for s, c in lc) % R
    return all(ev(a) * ev(b) % R == ev(c) for a, b, c in r1cs.constraints)


def domain_size_for(n_constraints: int, n_public: int) -> int:
    n = 1
    while n < n_constraints + n_public + 1:
        n *= 2
    return n
